"""CPU (gloo, world size 2 and 3): kernel-hash sharding of the scoring path.  Every rank
scores only its shard of the kernel columns; one all_gather of the [R][6] partials and a
fixed-order combine reproduce the single-process scores."""
import numpy as np
import pytest

import oracle as O
from _mp import run_world
from nvidia_resiliency_ext.straggler import synth


@pytest.mark.parametrize("ws", [2, 3])
def test_sharded_partials_reproduce_global_scores(ws):
    R, K, S, cap = 6, 40, 300, 256
    res = run_world(ws, "_shard_workers", "oracle_shard_partials", R=R, K=K, S=S, cap=cap)
    assert sum(res[r]["owned"] for r in range(ws)) == K      # the shards partition the kernels
    ns = O.gen_matrix(R, K, S)
    st = O.matrix_stats(ns.reshape(-1), R * K, S, 0, S, cap)
    gr, gi = O.scores(st["num"].reshape(R, K), st["med"].reshape(R, K), st["avg"].reshape(R, K))
    for r in range(ws):
        np.testing.assert_allclose(res[r]["rel"], gr, rtol=1e-13)
        np.testing.assert_allclose(res[r]["ind"], gi, rtol=1e-13)
    assert np.array_equal(O.stragglers(res[0]["rel"], 0.8), O.stragglers(gr, 0.8))


def test_shard_assignment_is_stable_and_balanced():
    names = synth.kernel_names(2048)
    for n in (2, 4, 8):
        parts = [set(synth.shard_kernels(names, n, g).tolist()) for g in range(n)]
        assert set().union(*parts) == set(range(2048))
        assert sum(len(p) for p in parts) == 2048
        assert min(len(p) for p in parts) > 0.8 * 2048 / n
    assert synth.kernel_hash("abc") == synth.kernel_hash("abc")
