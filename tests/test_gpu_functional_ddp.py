"""GPU functional test: a 2-rank DDP run (tests/func/ddp_straggler.py, the
shape of the reference's tests/straggler/func/ddp_test.py:172-245) with rank 1's wrapped
forward made 1.5x slower on the GPU; its log is checked the way the reference's
tests/straggler/func/check_log.py:29-51 checks it: the report count, the DETECTED RELATIVE
STRAGGLER GPU RANK= set == {1}, no individual stragglers, DONE."""
import os
import re
import socket
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _found(lines, pattern):
    # check_log.py:29-38 (_check_gpu_stragglers): the set of ranks on matching lines
    pat = re.compile(pattern)
    return {int(m.group(1)) for ln in lines for m in [pat.search(ln)] if m}


@pytest.mark.timeout(400)
def test_ddp_slow_rank_is_detected():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node=2",
           "--master-addr", "127.0.0.1", "--master-port", str(port),
           os.path.join(ROOT, "tests", "func", "ddp_straggler.py"),
           "--iters", "61", "--report-iter-interval", "20", "--slow-ranks", "1",
           "--slow-factor", "1.5"]
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=380)
    log = r.stdout.splitlines()
    assert r.returncode == 0, r.stderr[-4000:]
    print("\n".join(ln for ln in log if "STRAGGLER" in ln or "perf scores" in ln))
    assert any("DONE" in ln for ln in log)                              # check_log.py read_log_file
    assert len([ln for ln in log if "STRAGGLER REPORT" in ln]) == 3      # cmd_num_reports
    assert _found(log, r"DETECTED RELATIVE STRAGGLER GPU RANK=(\d+)") == {1}
    assert _found(log, r"DETECTED INDIVIDUAL STRAGGLER GPU RANK=(\d+)") == set()


@pytest.mark.timeout(500)
def test_gpt2_ddp_slow_rank_is_detected():
    """the same check on GPT-2 small (12 layers, d=768, ctx 1024, bf16
    autocast, fused AdamW; 2 ranks x 2 x 1024 tokens), rank 1's forward made 1.5x slower by the
    spin kernel sized to 10x the forward's captured kernel time (score 11/16 for rank 1, 1 for rank
    0; still below the 0.8 threshold SURVEY 8(d) sets should the model kernels' NUM x AVG weigh
    five times their NUM x MED, as duration spikes from the other process's time slices can make
    them on a shared GPU).  The forward's GEMM / attention / norm launches are captured and
    scored with it."""
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node=2",
           "--master-addr", "127.0.0.1", "--master-port", str(port),
           os.path.join(ROOT, "tests", "func", "ddp_straggler.py"),
           "--model", "gpt2", "--batch", "2", "--seq", "1024", "--iters", "31",
           "--report-iter-interval", "10", "--slow-ranks", "1", "--slow-factor", "1.5",
           "--spin-ratio", "10", "--base-iters", "5", "--threshold", "0.8"]
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=480)
    log = r.stdout.splitlines()
    assert r.returncode == 0, r.stderr[-4000:]
    print("\n".join(ln for ln in log if "STRAGGLER" in ln or "perf scores" in ln
                    or ln.startswith(("STEP MS", "SPIN", "CALIB"))))
    assert any("DONE" in ln for ln in log)
    assert len([ln for ln in log if "STRAGGLER REPORT" in ln]) == 3
    assert _found(log, r"DETECTED RELATIVE STRAGGLER GPU RANK=(\d+)") == {1}
    assert _found(log, r"DETECTED INDIVIDUAL STRAGGLER GPU RANK=(\d+)") == set()
    assert any(ln.startswith("STEP MS") for ln in log)
