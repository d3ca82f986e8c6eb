"""Reference-layout mirror (ViPT/lib) over the MI355X engine."""
