"""Per-tracker dispatch of RGB{D,T,E}/benchmark.py (the reference's time_cost dict; RGBE/benchmark.py:1-49,
RGBT/benchmark.py:1-38, RGBD/benchmark.py:1-63).

The reference changes directory into each tracker's folder and runs its test command with
os.system, recording wall seconds per tracker in ``time_cost``. Here every tracker this build
provides is a registry entry (working directory relative to the modality folder, argv); each runs
as a child process (so one tracker's GPU context never leaks into the next) and ``time_cost`` is
printed and written to ``time_cost.json``.
"""
from __future__ import annotations

import argparse
import json
import os
import subprocess
import sys
import time


def run(modality_dir: str, registry: dict, argv=None) -> dict:
    ap = argparse.ArgumentParser(description="Run the benchmark trackers and record wall time per tracker.")
    ap.add_argument("--trackers", nargs="*", default=None, help=f"subset of {sorted(registry)}")
    ap.add_argument("--out", default=None, help="time_cost JSON path (default <modality>/time_cost.json)")
    ap.add_argument("--dry_run", action="store_true", help="print the commands only")
    ap.add_argument("extra", nargs=argparse.REMAINDER, help="arguments appended to every tracker command")
    args = ap.parse_args(argv)
    names = args.trackers if args.trackers else list(registry)
    unknown = [n for n in names if n not in registry]
    if unknown:
        raise ValueError(f"unknown trackers {unknown}; available: {sorted(registry)}")
    extra = [a for a in (args.extra or []) if a != "--"]
    time_cost = {}
    for name in names:
        cwd, cmd = registry[name]
        wd = os.path.normpath(os.path.join(modality_dir, cwd))
        full = [sys.executable if c == "python" else c for c in cmd] + extra
        print(f"[benchmark] {name}: (cd {wd} && {' '.join(full)})", flush=True)
        if args.dry_run:
            continue
        begin = time.time()
        rc = subprocess.call(full, cwd=wd)
        time_cost[name] = time.time() - begin
        if rc != 0:
            print(f"[benchmark] {name} exited with {rc}", flush=True)
    print(time_cost)
    if not args.dry_run:
        with open(args.out or os.path.join(modality_dir, "time_cost.json"), "w") as f:
            json.dump(time_cost, f, indent=1)
    return time_cost
