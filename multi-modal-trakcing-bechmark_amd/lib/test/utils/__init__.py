from .params import TrackerParams  # noqa: F401
