"""CPU: pin the oracle to the reference's own outputs (tests/golden, made by
tests/golden/make_golden.py from the reference).  If these pass, the oracle used by
the GPU parity tests is the reference's semantics, bit for bit."""
import json
import math
import os

import numpy as np
import pytest

import oracle as O
import oracle_report as OR

HERE = os.path.dirname(os.path.abspath(__file__))
GOLD = os.path.join(HERE, "golden")

import sys  # noqa: E402

sys.path.insert(0, GOLD)
import scenarios as SC  # noqa: E402


def _load(name):
    with open(os.path.join(GOLD, name)) as f:
        return json.load(f)


def oracle_stats_fn(ns_u32, cap=8192):
    us = O.ns_to_us(np.asarray(ns_u32, np.uint32))
    kept = O.ring_linearize(us, cap)
    st = O.compute_stats(kept)
    return (st.num_calls, np.float32(st.min), np.float32(st.max), np.float32(st.median),
            np.float32(st.avg), np.float32(st.stddev))


def _bits(x):
    return int(np.float32(x).view(np.uint32))


def test_compute_stats_kat_bit_exact():
    kat = _load("compute_stats_kat.json")
    assert len(kat["cases"]) >= 10
    for c in kat["cases"]:
        if "gen" in c:
            g = c["gen"]
            m = O.gen_matrix(g["R"], g["K"], g["S"], seed=g["seed"],
                             straggler=np.array(g["straggler"], np.uint8))
            ns = m[g["r"], g["k"]]
        else:
            ns = np.array(c["ns"], np.uint64).astype(np.uint32)
        r = oracle_stats_fn(ns, c["cap"])
        got = [int(r[0])] + [_bits(v) for v in r[1:]]
        assert got == c["expect"], c["name"]


def test_duration_conversion_bit_exact():
    conv = _load("compute_stats_kat.json")["conversion"]
    us = O.ns_to_us(np.array(conv["ns"], np.uint64))
    assert [_bits(v) for v in us] == conv["us_bits"]
    assert [_bits(O.lib().oracle_ns_to_us(n)) for n in conv["ns"]] == conv["us_bits"]


def test_ring_semantics_match_circular_buffer():
    # CircularBuffer.h:53-69: capacity 4, pushes 1..6 -> linearize [3, 4, 5, 6]
    out = O.ring_linearize(np.arange(1, 7, dtype=np.float32), 4)
    assert out.tolist() == [3.0, 4.0, 5.0, 6.0]
    st = O.compute_stats(out)
    assert st.median == 4.5 and abs(st.stddev - 1.11803) < 1e-5


def _gen(R, K, S, seed, strag):
    return O.gen_matrix(R, K, S, seed=seed, straggler=strag)


def _fixture_sections(fx, t, r):
    secs = fx["section_summaries"][t][r]
    return {n: {k: (v if k == "NUM" else float.fromhex(v)) for k, v in s.items()}
            for n, s in secs.items()}


def _assert_scores_equal(got: dict, want: dict, where: str, exact=True, rtol=0.0):
    assert set(got.keys()) == set(want.keys()), (where, got.keys(), want.keys())
    for k, v in want.items():
        g = got[k]
        if isinstance(v, dict):
            _assert_scores_equal(g, v, f"{where}/{k}", exact, rtol)
            assert list(g.keys()) == list(v.keys()), (where, "order")
        else:
            w = SC.decode_value(v)
            gv = SC.decode_value(g) if isinstance(g, str) else g
            if math.isnan(w):
                assert math.isnan(gv), (where, k)
            elif exact:
                assert gv == w, (where, k, gv, w)
            else:
                assert abs(gv - w) <= rtol * abs(w), (where, k, gv, w)


SCEN = sorted(SC.SCENARIOS)


@pytest.mark.parametrize("scname", SCEN)
def test_oracle_report_matches_reference(scname):
    fx = _load(f"report_{scname}.json")
    sc = SC.SCENARIOS[scname]
    ws = sc["ws"]
    world = OR.SimWorld(ws, sc["scores"], sc["gather"], [f"node{r}" for r in range(ws)])
    prev_gathers = 0
    for t in range(sc["reports"]):
        sections, kernels = [], []
        for r in range(ws):
            _, ker = SC.build_rank_inputs(sc, r, t, _gen, oracle_stats_fn,
                                          OR.section_summary_torch_semantics)
            # oracle computeStats regenerates the reference's kernel summaries exactly
            assert SC.summaries_digest({}, ker) == fx["kernel_summary_sha256"][t][r], (t, r)
            sec = _fixture_sections(fx, t, r)
            # the numpy restatement of the torch section statistics, within 1 ulp
            _, sec_np_k = None, None
            mine = {n: OR.section_summary_torch_semantics(
                SC.section_timings(sc, r, t, int(n[len("section"):]))) for n in sec}
            for n in sec:
                for k in ("MIN", "MAX", "MED", "NUM"):
                    assert mine[n][k] == sec[n][k], (n, k)
                for k in ("AVG", "STD"):
                    a, b = mine[n][k], sec[n][k]
                    assert (math.isnan(a) and math.isnan(b)) or abs(a - b) <= 4e-16 * abs(b)
            sections.append(sec)
            kernels.append(ker)
        outs = world.generate_report(sections, kernels)
        for r in range(ws):
            want = fx["reports"][t][r]
            got = outs[r]
            if want is None:
                assert got is None
                continue
            enc = SC.encode_report(got)
            for f in SC.REPORT_FIELDS:
                _assert_scores_equal(enc[f], want[f], f"{scname}/t{t}/r{r}/{f}")
            assert enc["rank_to_node"] == want["rank_to_node"]
            assert enc["rank"] == want["rank"] and enc["gather_on_rank0"] == want["gather_on_rank0"]
        # all_gather_object calls: names (NameMapper) + rank->node (first report, gather)
        calls = world.mapper.gathers - prev_gathers + (1 if (t == 0 and sc["gather"]) else 0)
        prev_gathers = world.mapper.gathers
        assert all(c == calls for c in fx["all_gather_object_calls"][t]), (t, calls)
    if sc["gather"] or "relative_perf_scores" in sc["scores"]:
        assert world.mapper.kernel_name_to_id == fx["name_mapper"]["kernel"]
        assert world.mapper.section_name_to_id == fx["name_mapper"]["section"]


def test_ns_to_us_reciprocal_multiply_identity():
    # the kernels convert ns -> us as f32(f64(f32(ns)) * RN(1/1000)) (nvrx_common.h ns_to_us);
    # that equals the reference's correctly rounded f32(ns) / 1000.0f (CuptiProfiler.cpp:187)
    # for every u32 -- checked exhaustively offline; here 2^24 random values plus the edges
    rng = np.random.default_rng(187)
    x = np.concatenate([
        rng.integers(0, 2**32, size=1 << 24, dtype=np.uint64).astype(np.uint32),
        np.arange(0, 1 << 16, dtype=np.uint32),
        (np.uint64(1) << np.arange(32, dtype=np.uint64)).astype(np.uint32),
        np.array([2**24 - 1, 2**24 + 1, 2**24 + 3, 2**32 - 1, 2**31 - 1, 999, 1000, 1001],
                 dtype=np.uint32)])
    f = x.astype(np.float32)
    ref = f / np.float32(1000.0)
    got = (f.astype(np.float64) * (1.0 / 1000.0)).astype(np.float32)
    assert np.array_equal(ref.view(np.uint32), got.view(np.uint32))


def test_wide_duration_kat_bit_exact():
    """u64 durations of 2^32 ns and more: the reference's own conversion
    (end - start) / 1000.0f and computeStats over it (compute_stats_wide_kat.json, made from the
    reference build), reproduced by the oracle's conversion, and by the duration keys: decoding a
    key gives back exactly the f32(ns) the reference divides."""
    kat = _load("compute_stats_wide_kat.json")
    conv = kat["conversion"]
    ns = np.array(conv["ns"], np.uint64)
    assert [_bits(v) for v in O.ns_to_us(ns)] == conv["us_bits"]
    assert [_bits(O.lib().oracle_ns_to_us(int(n))) for n in conv["ns"]] == conv["us_bits"]
    assert [_bits(v) for v in O.key_to_us(O.duration_key(ns))] == conv["us_bits"]
    assert len(kat["cases"]) >= 10
    for c in kat["cases"]:
        x = np.array(c["ns"], np.uint64)
        st = O.compute_stats(O.ring_linearize(O.ns_to_us(x), c["cap"]))
        got = [int(st.num_calls)] + [_bits(v) for v in (st.min, st.max, st.median, st.avg, st.stddev)]
        assert got == c["expect"], c["name"]
        # the key route the HIP kernels take: keys -> f32 us, same bits
        kst = O.compute_stats(O.ring_linearize(O.key_to_us(O.duration_key(x)), c["cap"]))
        kgot = [int(kst.num_calls)] + [_bits(v) for v in (kst.min, kst.max, kst.median, kst.avg, kst.stddev)]
        assert kgot == c["expect"], c["name"]
