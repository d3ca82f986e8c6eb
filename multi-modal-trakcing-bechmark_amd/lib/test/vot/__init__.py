"""VOT / TraX integration of the tracker (ViPT/lib/test/vot), SURVEY §8 f1."""
