"""FAST-mode AVG / STD parity bar shared by the record-stream tests.

Every (stream, slot) statistic is either bit-exact with the reference's computeStats (sequential
f32 sums over the sorted samples: the one-lane-per-bucket paths) or within the FAST bar of the
exact f64 moments of the retained integer-ns samples: AVG 2.5e-7, STD 1e-6 relative.  Buckets of
<= LANE_EXACT records are always bit-exact."""
import numpy as np

AVG_RTOL = 2.5e-7
KEY_WIDE = 0xE0000000


def key_values(keys):
    """float64 duration values (ns) behind u32 duration keys, as the FAST kernels average them:
    the integers while every key is below KEY_WIDE, else the decoded f32(ns) values."""
    import oracle as O

    k = np.asarray(keys, np.uint32)
    if k.size and int(k.max()) >= KEY_WIDE:
        return O.key_to_f32(k).astype(np.float64)
    return k.astype(np.float64)
STD_RTOL = 1e-6
LANE_EXACT = 128  # the lane classes (<= 128 records, nvrx_straggler.h) are bit-exact


def check_avg_std(g_avg, g_std, ref, xmean, xstd, tag=""):
    """g_*: GPU float32 arrays; ref: oracle records_stats dict; xmean / xstd: records_moments."""
    num = ref["num"]
    present = num > 0
    for f, g, x, tol in (("avg", g_avg, xmean, AVG_RTOL), ("std", g_std, xstd, STD_RTOL)):
        g = np.asarray(g)
        same = g.view(np.uint32) == ref[f].view(np.uint32)
        short = present & (num <= LANE_EXACT)
        bad = np.count_nonzero(short & ~same)
        assert bad == 0, f"{tag}: {f} not bit-exact in {bad} buckets of <= {LANE_EXACT} records"
        err = np.abs(g.astype(np.float64) - x) / np.where(x != 0, np.abs(x), 1.0)
        ok = same | (err <= tol)
        bad = np.count_nonzero(present & ~ok)
        worst = float(np.max(np.where(present & ~same, err, 0.0))) if present.any() else 0.0
        assert bad == 0, f"{tag}: {f} outside the FAST bar {tol} in {bad} buckets (worst {worst:.3e})"
