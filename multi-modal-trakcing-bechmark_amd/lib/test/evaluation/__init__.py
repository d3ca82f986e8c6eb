from .data import Sequence  # noqa: F401
from .tracker import Tracker, trackerlist  # noqa: F401
