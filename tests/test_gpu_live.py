"""GPU: configs[4] live capture end to end -- the GPT-2 small DDP loop (12 layers, d=768, ctx
1024; tools/live_gpt2.py, RCCL world of 1) under the Detector, kernel dispatches captured into
the device record log; the report's per-kernel statistics are checked bit for bit against the
oracle's ring-push + computeStats restatement over the very records captured, and every report
window holds exactly its steps' launches.  The 2-rank DDP run of the same model with a slowed
rank is tests/test_gpu_functional_ddp.py::test_gpt2_ddp_slow_rank_is_detected."""
import json
import os
import random
import subprocess
import sys

import numpy as np
import pytest

import oracle as O

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_live_gpt2_capture_stats_match_oracle(tmp_path):
    dump = tmp_path / "live.npz"
    out = tmp_path / "live.json"
    env = dict(os.environ, MASTER_ADDR="127.0.0.1", MASTER_PORT=str(random.randint(20000, 40000)),
               RANK="0", WORLD_SIZE="1", LOCAL_RANK="0")
    cmd = [sys.executable, os.path.join(ROOT, "tools", "live_gpt2.py"), "--layers", "12",
           "--batch", "4", "--seq", "1024", "--warmup", "2", "--base-steps", "5", "--steps", "10",
           "--report-every", "5", "--count-check", "--dump", str(dump), "--out", str(out)]
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=600, env=env)
    assert r.returncode == 0, r.stderr[-4000:]
    res = json.loads(out.read_text())
    print({k: res[k] for k in ("workload", "step_ms_without_detector", "step_ms_with_detector",
                               "detector_overhead_pct", "report_ms_median", "records_per_report",
                               "kernel_keys")})
    assert res["capture"] is True
    assert res["kernel_keys"] > 50 and res["records_per_report"] > 1000
    assert res["gpu_relative_perf_scores"] == {"0": 1.0} or res["gpu_relative_perf_scores"] == {0: 1.0}
    # completeness (no explicit flush before the reports): every 5-step window holds exactly
    # 5 x each key's launches of a one-step window -- nothing lost, nothing carried over
    step = res["step_counts"]
    assert step and len(res["window_counts"]) == 2
    for w in res["window_counts"]:
        assert w == {k: 5 * n for k, n in step.items()}, \
            {k: (w.get(k), 5 * step.get(k, 0)) for k in set(w) | set(step) if w.get(k) != 5 * step.get(k, 0)}

    d = np.load(dump)
    slots, ns = d["slots"], d["ns"]
    # every captured step contributes the same kernels: 5 steps per window
    nslots = int(slots.max()) + 1
    recs = np.stack([slots, ns], axis=1).astype(np.uint32)
    st = O.records_stats(recs, np.array([0, len(recs)], np.int64), nslots, cap=int(d["cap"]))
    slot_name = dict(zip(d["slot_ids"].tolist(), d["slot_names"].tolist()))
    want = {slot_name[s]: s for s in range(nslots) if st["num"][s] > 0}
    names = d["names"].tolist()
    assert sorted(want) == names  # name-sorted, every kernel with records
    for i, n in enumerate(names):
        s = want[n]
        for f in ("num", "min", "max", "med", "avg", "std"):
            a, b = d[f][i], st[f][s]
            assert a.tobytes() == b.tobytes(), (n, f, a, b)
