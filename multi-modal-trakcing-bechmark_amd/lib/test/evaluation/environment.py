"""env_settings(): project / result paths (ViPT/lib/test/evaluation/environment.py; local.py)."""
import os


class EnvSettings:
    def __init__(self):
        prj = os.path.abspath(os.path.join(os.path.dirname(__file__), '..', '..', '..'))
        self.prj_dir = os.environ.get("MMTRACK_PRJ_DIR", prj)
        self.save_dir = os.environ.get("MMTRACK_SAVE_DIR", os.path.join(self.prj_dir, "output"))
        self.results_path = os.path.join(self.save_dir, 'test', 'tracking_results')
        self.result_plot_path = os.path.join(self.save_dir, 'test', 'result_plots')
        self.network_path = os.path.join(self.save_dir, 'test', 'networks')


def env_settings():
    return EnvSettings()
