"""VOT integration handle (ViPT/lib/test/vot/vot.py:8-111): region(), frame(), report(), quit().

The reference talks TraX (``trax.Server``).  trax 3.0.3 is not installed in this image, so the handle
takes an optional ``source``: any object with ``region() -> Rectangle``, ``frame() -> path | [color,
aux] | None`` and ``report(region, properties)`` -- ``SequenceSource`` replays a dataset sequence and
keeps the reports (the offline / test client).  Without a source the handle needs trax and raises the
reference's exception text when it is missing.
"""
import collections

import numpy as np

Rectangle = collections.namedtuple('Rectangle', ['x', 'y', 'width', 'height'])
Point = collections.namedtuple('Point', ['x', 'y'])
Polygon = collections.namedtuple('Polygon', ['points'])

_CHANNELS = {None: ['color'], 'rgbd': ['color', 'depth'], 'rgbt': ['color', 'ir'], 'ir': ['ir']}


class SequenceSource:
    """A TraX client stand-in over one sequence: frames[i] is an image path or a [color, aux] pair,
    region is the first-frame rectangle; report() stores (region, properties) per tracked frame."""

    def __init__(self, region, frames):
        self._region = Rectangle(*[float(v) for v in region])
        self._frames = list(frames)
        self._next = 0
        self.reports = []

    def region(self):
        return self._region

    def frame(self):
        if self._next >= len(self._frames):
            return None
        f = self._frames[self._next]
        self._next += 1
        return f

    def report(self, region, properties):
        self.reports.append((region, dict(properties)))


class VOT(object):
    """Base class for Python VOT integration (vot.py:22-111)."""

    def __init__(self, region_format, channels=None, source=None):
        self._source = None   # set first: a failed construction must still quit() cleanly from __del__
        if channels not in _CHANNELS:
            raise Exception('Illegal configuration {}.'.format(channels))
        self.channels = _CHANNELS[channels]
        if source is None:
            try:
                import trax
            except ImportError:
                raise Exception('TraX support not found. Please add trax module to Python path.')
            source = _TraxSource(trax, region_format, self.channels)
        elif region_format != 'rectangle':
            raise Exception('only the rectangle region format is served offline')
        self._source = source
        self._region = source.region()
        self._image = source.frame()

    def region(self):
        return self._region

    def report(self, region, confidence=None):
        assert isinstance(region, (Rectangle, Polygon, np.ndarray))
        properties = {}
        if confidence is not None:
            properties['confidence'] = confidence
        self._source.report(region, properties)

    def frame(self):
        if hasattr(self, '_image'):
            image = self._image
            del self._image
            return image
        return self._source.frame()

    def quit(self):
        q = getattr(getattr(self, '_source', None), 'quit', None)
        if q is not None:
            q()

    def __del__(self):
        self.quit()


class _TraxSource:
    """The reference's TraX server exchange (vot.py:31-111)."""

    def __init__(self, trax, region_format, channels):
        self._trax_mod = trax
        self._trax = trax.Server([region_format], [trax.Image.PATH], channels, customMetadata=dict(vot="python"))
        request = self._trax.wait()
        assert request.type == 'initialize'
        if isinstance(request.region, trax.Polygon):
            self._region = Polygon([Point(x[0], x[1]) for x in request.region])
        elif isinstance(request.region, trax.Mask):
            self._region = request.region.array(True)
        else:
            self._region = Rectangle(*request.region.bounds())
        image = [x.path() for k, x in request.image.items()]
        self._first = image[0] if len(image) == 1 else image
        self._trax.status(request.region)

    def region(self):
        return self._region

    def frame(self):
        if self._first is not None:
            f, self._first = self._first, None
            return f
        request = self._trax.wait()
        if request.type == 'frame':
            image = [x.path() for k, x in request.image.items()]
            return image[0] if len(image) == 1 else image
        return None

    def report(self, region, properties):
        trax = self._trax_mod
        if isinstance(region, Polygon):
            tregion = trax.Polygon.create([(x.x, x.y) for x in region.points])
        elif isinstance(region, np.ndarray):
            tregion = trax.Mask.create(region)
        else:
            tregion = trax.Rectangle.create(region.x, region.y, region.width, region.height)
        self._trax.status(tregion, properties)

    def quit(self):
        self._trax.quit()
