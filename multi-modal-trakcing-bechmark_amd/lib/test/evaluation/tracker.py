"""Tracker wrapper (ViPT/lib/test/evaluation/tracker.py:28-311): dynamic import of
lib.test.tracker.<name>.get_tracker_class() and lib.test.parameter.<name>.parameters(<yaml>)."""
import importlib
import os
import time
from collections import OrderedDict

from lib.test.evaluation.environment import env_settings


def trackerlist(name, parameter_name, dataset_name, run_ids=None, display_name=None, result_only=False):
    if run_ids is None or isinstance(run_ids, int):
        run_ids = [run_ids]
    return [Tracker(name, parameter_name, dataset_name, run_id, display_name, result_only) for run_id in run_ids]


class Tracker:
    def __init__(self, name: str, parameter_name: str, dataset_name: str, run_id: int = None,
                 display_name: str = None, result_only=False):
        assert run_id is None or isinstance(run_id, int)
        self.name = name
        self.parameter_name = parameter_name
        self.dataset_name = dataset_name
        self.run_id = run_id
        self.display_name = display_name
        env = env_settings()
        if self.run_id is None:
            self.results_dir = '{}/{}/{}'.format(env.results_path, self.name, self.parameter_name)
        else:
            self.results_dir = '{}/{}/{}_{:03d}'.format(env.results_path, self.name, self.parameter_name, self.run_id)
        if result_only:
            self.results_dir = '{}/{}'.format(env.results_path, self.name)
        path = os.path.abspath(os.path.join(os.path.dirname(__file__), '..', 'tracker', '%s.py' % self.name))
        if os.path.isfile(path):
            self.tracker_class = importlib.import_module('lib.test.tracker.{}'.format(self.name)).get_tracker_class()
        else:
            self.tracker_class = None
        self.param_overrides = {}

    def create_tracker(self, params):
        return self.tracker_class(params)

    def get_parameters(self):
        param_module = importlib.import_module('lib.test.parameter.{}'.format(self.name))
        params = param_module.parameters(self.parameter_name)
        for k, v in self.param_overrides.items():
            setattr(params, k, v)
        return params

    def run_sequence(self, seq, debug=None):
        params = self.get_parameters()
        params.debug = getattr(params, 'debug', 0) if debug is None else debug
        tracker = self.create_tracker(params)
        return self._track_sequence(tracker, seq, seq.init_info())

    def _track_sequence(self, tracker, seq, init_info):
        """tracker.py:91-164: per-frame time includes reading the frame, as in the reference."""
        output = {'target_bbox': [], 'time': [], 'all_scores': []}
        image = seq.image(0)
        start_time = time.time()
        out = tracker.initialize(image, init_info) or {}
        prev_output = OrderedDict(out)
        output['target_bbox'].append(init_info.get('init_bbox'))
        output['time'].append(time.time() - start_time)
        output['all_scores'].append(1)
        for frame_num in range(1, len(seq)):
            image = seq.image(frame_num)
            start_time = time.time()
            info = seq.frame_info(frame_num)
            info['previous_output'] = prev_output
            out = tracker.track(image, info)
            prev_output = OrderedDict(out)
            output['target_bbox'].append(out['target_bbox'])
            output['time'].append(time.time() - start_time)
            output['all_scores'].append(out.get('best_score', None))
        if any(s is None for s in output['all_scores']):
            output.pop('all_scores')
        return output
