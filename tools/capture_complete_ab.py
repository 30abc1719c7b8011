"""Capture completeness A/B under host load (not part of the library): runs the two-stream,
8-interval Detector case of tests/test_gpu_capture_complete.py in a child process per mode, with
every host core kept busy, and prints per mode how many launches each report missed or carried
over.  Modes: the default (callback delivery, flush counted at enqueue), the uncounted quiet-
period flush (NVRX_CAPTURE_MARKING=0: the round-4 default), and buffer delivery (counted).
Output: one JSON line per mode (and --out FILE, a JSON list)."""
import argparse
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tests"))

import test_gpu_capture_complete as T  # noqa: E402

MODES = {
    "callback_counted_flush": {},
    "callback_quiet_flush": {"NVRX_CAPTURE_MARKING": "0"},
    "buffer_counted_flush": {"NVRX_CAPTURE_DELIVERY": "buffer"},
}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--hogs", type=int, default=32)
    ap.add_argument("--repeats", type=int, default=2)
    ap.add_argument("--out", default=None)
    a = ap.parse_args()
    rows = []
    for rep in range(a.repeats):
        for mode, env in MODES.items():
            hogs = T._busy(a.hogs)
            try:
                out = T._child(T.LOADED, env=env)
            finally:
                for h in hogs:
                    h.kill()
                for h in hogs:
                    h.wait()
            missed = carried = 0
            bad = []
            for i, (g, w) in enumerate(zip(out["got"], out["want"])):
                for k in set(g) | set(w):
                    d = g.get(k, 0) - w.get(k, 0)
                    missed += max(0, -d)
                    carried += max(0, d)
                    if d:
                        bad.append(i)
            row = {"mode": mode, "repeat": rep, "hogs": a.hogs,
                   "launches": sum(sum(w.values()) for w in out["want"]),
                   "missed": missed, "carried_over": carried, "bad_intervals": sorted(set(bad)),
                   **{k: out[k] for k in ("counted", "quiet", "timeouts", "abandoned", "enqueues",
                                          "flush_ms")}}
            rows.append(row)
            print(json.dumps(row), flush=True)
    if a.out:
        with open(a.out, "w") as f:
            json.dump(rows, f, indent=1)


if __name__ == "__main__":
    main()
