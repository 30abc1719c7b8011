"""bench.py's multi-rank launcher: `python bench.py --gpus N` (no WORLD_SIZE) starts
torch.distributed.run with N ranks of itself as a child process, and rank 0 prints the one JSON
line with n_gpus = N (VERDICT r01 "next 2").

CPU: --dry-run (launcher + gloo rendezvous, no GPU work).  GPU: the real 2-rank rehearsal on the
box's one GPU with the partials exchanged over gloo (NVRX_BENCH_BACKEND=gloo), a reduced run."""
import json
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
BENCH = os.path.join(ROOT, "bench.py")


def _run(args, timeout):
    env = {k: v for k, v in os.environ.items()
           if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT")}
    env["NVRX_BENCH_BACKEND"] = "gloo"
    p = subprocess.run([sys.executable, BENCH] + args, capture_output=True, text=True, env=env,
                       timeout=timeout)
    assert p.returncode == 0, p.stderr[-3000:]
    lines = [ln for ln in p.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, p.stdout  # rank 0 only
    return json.loads(lines[0])


def test_launcher_two_ranks_dry_run():
    line = _run(["--gpus", "2", "--dry-run"], timeout=240)
    assert line == {"dry_run": True, "n_gpus": 2, "world_size": 2, "backend": "gloo"}


@pytest.mark.gpu
@pytest.mark.timeout(400)
def test_launcher_two_ranks_gloo_rehearsal():
    line = _run(["--gpus", "2", "--steps", "3", "--warmup", "1", "--no-zipf", "--no-cpu-baseline"],
                timeout=380)
    assert line["n_gpus"] == 2
    assert line["config"]["world_size"] == 2 and line["config"]["backend"] == "gloo"
    assert line["config"]["kernels_total"] == 4096
    assert line["straggler_sets_exact"] is True
    assert line["latency_4096_ranks"]["straggler_sets_exact"] is True
    assert 0 < line["roofline"]["frac"] < 1.5


def test_launcher_four_ranks_dry_run():
    line = _run(["--gpus", "4", "--dry-run"], timeout=300)
    assert line == {"dry_run": True, "n_gpus": 4, "world_size": 4, "backend": "gloo"}


@pytest.mark.gpu
@pytest.mark.timeout(600)
def test_launcher_four_ranks_gloo_rehearsal():
    # the N > 1 line as the driver's 8-GPU node will print it, rehearsed with
    # 4 ranks on the one GPU over gloo: the world size the process group reports, the kernel
    # shard of every rank, and exact straggler sets (on every rank) for all three legs
    line = _run(["--gpus", "4", "--steps", "3", "--warmup", "1", "--no-cpu-baseline"], timeout=580)
    cfg = line["config"]
    assert line["n_gpus"] == 4 and cfg["world_size"] == 4 and cfg["world_size_reported"] == 4
    assert cfg["backend"] == "gloo" and cfg["kernels_total"] == 4 * 2048
    assert sum(cfg["kernels_per_rank"]) == 4 * 2048 and len(cfg["kernels_per_rank"]) == 4
    assert min(cfg["kernels_per_rank"]) > 0
    assert line["straggler_sets_exact"] is True
    lat, zipf = line["latency_4096_ranks"], line["zipf_16384_ranks"]
    assert lat["straggler_sets_exact"] is True and sum(lat["kernels_per_rank"]) == 2048
    assert zipf["straggler_sets_exact"] is True and sum(zipf["kernels_per_rank"]) == 2048
    # every rank runs the same launch mode -- reports two in flight, each
    # one's statistics, partials and combine as graphs, only the all_gather eager -- and the
    # strong-scaled legs report what one GPU reports (f64 combine order aside)
    for leg in (cfg, lat, zipf):
        labels = leg["launch_per_rank"]
        assert len(labels) == 4 and len(set(labels)) == 1, labels
        assert labels[0].startswith("hip_graph: reports two in flight"), labels
        assert labels[0].endswith("(statistics | score partials | eager all_gather | combine)"), labels
    # configs[1] per GPU (4.3 GB of samples per report): each report on its own stream
    assert cfg["launch_per_rank"][0].startswith("hip_graph: reports two in flight, each on its own stream")
    # every point also carries the one-report-at-a-time launch mode's time,
    # labelled (on N > 1: partials | eager all_gather | combine)
    want = "hip_graph: statistics | score partials | eager all_gather | combine"
    gp = line["graph_phases"]
    assert gp["launch_per_rank"] == [want] * 4 and gp["straggler_sets_exact"] is True
    assert line["ms_per_step_graph_phases"] > 0
    one = _run(["--gpus", "1", "--steps", "3", "--warmup", "1", "--no-cpu-baseline"], timeout=580)
    alt = "hip_graph: reports two in flight, each on its own stream"
    assert one["zipf_16384_ranks"]["launch_per_rank"] == [alt] and one["config"]["launch"] == alt
    # configs[2] (34 GB of samples per report): whole reports on one stream (PIPE_ALT_MAX_BYTES)
    assert one["latency_4096_ranks"]["launch_per_rank"] == ["hip_graph: whole reports, two in flight"]
    assert one["graph_phases"]["launch_per_rank"] == ["hip_graph: statistics | rest"]
    assert one["graph_phases"]["straggler_sets_exact"] is True
    assert one["ms_per_step_graph_phases"] > 0
    for leg in ("latency_4096_ranks", "zipf_16384_ranks"):
        a, b = line[leg]["scores"], one[leg]["scores"]
        assert a["stragglers_rel"] == b["stragglers_rel"], leg
        for f in ("rel_sum", "ind_sum"):
            assert abs(a[f] - b[f]) <= 1e-9 * abs(b[f]), (leg, f, a[f], b[f])
