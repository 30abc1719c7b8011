"""Rank workers for the multi-process ReportGenerator tests (run inside tests/_mp.run_world).

The KAT workers restate the reference's own unit tests
(tests/straggler/unit/test_relative_gpu_scores.py, test_individual_gpu_scores.py,
test_name_mapper.py, test_data_shared.py) against this build's HIP-backed ReportGenerator.
"""
import json
import os
import random

import numpy as np


def _S():
    from nvidia_resiliency_ext import straggler

    return straggler


def get_summary(timings):
    """Same construction as the reference tests' _get_summary (numpy float64 stats)."""
    S = _S().Statistic
    timings = np.asarray(timings, dtype=np.float64)
    return {S.MIN: np.min(timings), S.MAX: np.max(timings), S.MED: np.median(timings),
            S.AVG: np.mean(timings),
            S.STD: (np.std(timings).item() if len(timings) > 1 else float("nan")),
            S.NUM: len(timings)}


def _enc(rep):
    import scenarios as SC

    return SC.encode_report(rep)


# ---------------------------------------------------------------- relative scores
def rel_scores(rank, ws, gather_on_rank0):
    random.seed(rank)
    rg = _S().reporting.ReportGenerator(['relative_perf_scores'], gather_on_rank0=gather_on_rank0,
                                        node_name=f'testnode{rank}')
    ks = {
        'kernel0': get_summary((rank + 1) * np.array([1.0, 1.0, 2.0])),
        'kernel1': get_summary((rank + 1) * np.array([2.0, 2.0, 3.0])),
        'ncclDevKernel_AllReduce_Sum': get_summary((ws - rank) * np.array([10.0, 20.0, 30.0])),
    }
    names = list(ks)
    random.shuffle(names)
    return _enc(rg.generate_report({}, kernel_summaries={n: ks[n] for n in names}))


def rel_some_common(rank, ws):
    rg = _S().reporting.ReportGenerator(['relative_perf_scores'], gather_on_rank0=True,
                                        node_name=f'testnode{rank}')
    ks = {'kernel_common': get_summary((rank + 1) * np.array([1.0, 1.0, 2.0])),
          f'kernel_only_on_rank{rank}': get_summary((rank + 1) * np.array([2.0, 2.0, 3.0]))}
    return _enc(rg.generate_report({}, kernel_summaries=ks))


def rel_no_common(rank, ws, ranks_with_unique_kernels=(), ranks_without_kernels=()):
    rg = _S().reporting.ReportGenerator(['relative_perf_scores'], gather_on_rank0=True,
                                        node_name=f'testnode{rank}')
    if rank in ranks_with_unique_kernels:
        ks = {f'rank_specific_kernel{rank}': get_summary(np.array([99.0, 99.0, 99.0]))}
    elif rank in ranks_without_kernels:
        ks = {}
    else:
        ks = {'kernel_common0': get_summary((rank + 1) * np.array([1.0, 1.0, 2.0])),
              'kernel_common1': get_summary((rank + 1) * np.array([2.0, 2.0, 3.0]))}
    return _enc(rg.generate_report({}, kernel_summaries=ks))


# ---------------------------------------------------------------- individual scores
def indiv_scores(rank, ws, gather_on_rank0):
    rg = _S().reporting.ReportGenerator(['individual_perf_scores'],
                                        gather_on_rank0=gather_on_rank0,
                                        node_name=f'testnode{rank}')
    rg.generate_report({}, kernel_summaries={
        'kernel0': get_summary(np.array([1.0, 1.0, 2.0])),
        'kernel1': get_summary(np.array([2.0, 2.0, 3.0]))})
    rep = rg.generate_report({}, kernel_summaries={
        'kernel0': get_summary((rank + 1) * np.array([1.0, 1.0, 2.0])),
        'kernel1': get_summary((rank + 1) * np.array([2.0, 2.0, 3.0]))})
    return _enc(rep)


# ---------------------------------------------------------------- name mapper
def mapping_consistency(rank, ws, gather_on_rank0):
    rg = _S().reporting.ReportGenerator(['relative_perf_scores'], gather_on_rank0=gather_on_rank0,
                                        node_name=f'testnode{rank}')
    rg.generate_report(section_summaries={f'initial_section_rank{rank}': get_summary([1.0])},
                       kernel_summaries={f'initial_kernel_rank{rank}': get_summary([1.0])})
    if rank == 0:
        ks = {'rank0_only': get_summary([1.0]), 'k1': get_summary([4.0]), 'k2': get_summary([6.0])}
        ss = {'rank0_only': get_summary([1.0]), 's1': get_summary([4.0]), 's2': get_summary([6.0])}
    else:
        ks = {'k2': get_summary([3.0]), 'k1': get_summary([2.0]), 'rank1_only': get_summary([1.0])}
        ss = {'s2': get_summary([3.0]), 's1': get_summary([2.0]), 'rank1_only': get_summary([1.0])}
    rep = rg.generate_report(section_summaries=ss, kernel_summaries=ks)
    m = rg.name_mapper
    return dict(report=_enc(rep), kernel_counter=m.kernel_counter,
                section_counter=m.section_counter, kernel_ids=m.kernel_name_to_id,
                section_ids=m.section_name_to_id)


def all_gather_counts(rank, ws):
    """test_data_shared.py:47-100: number of all_gather_object calls per report."""
    from unittest.mock import patch

    import torch

    orig = torch.distributed.all_gather_object
    rg = _S().reporting.ReportGenerator(['relative_perf_scores'], gather_on_rank0=True,
                                        node_name=f'testnode{rank}')
    post = '_' * 1024
    ks = {f'kernel{k}_{post}': get_summary(np.ones(8)) for k in range(4096)}
    new = {f'new_kernel{k}_{post}': get_summary(np.ones(8)) for k in range(4096)}
    new.update(ks)
    counts = []
    for summ in (ks, ks, new, new,
                 ({'the_latest_kernel_rank0': get_summary(np.ones(8))} if rank == 0 else ks)):
        with patch('torch.distributed.all_gather_object', wraps=orig) as m:
            rg.generate_report({}, kernel_summaries=summ)
            counts.append(m.call_count)
    return counts


# ---------------------------------------------------------------- golden scenarios
def golden_scenario(rank, ws, scname, stats_source="oracle"):
    import scenarios as SC

    import oracle as O
    import oracle_report as OR

    straggler = _S()
    here = os.path.dirname(os.path.abspath(__file__))
    with open(os.path.join(here, "golden", f"report_{scname}.json")) as f:
        fx = json.load(f)
    sc = SC.SCENARIOS[scname]
    if stats_source == "oracle":
        def stats_fn(ns, cap=8192):
            st = O.compute_stats(O.ring_linearize(O.ns_to_us(np.asarray(ns, np.uint32)), cap))
            return (st.num_calls, np.float32(st.min), np.float32(st.max), np.float32(st.median),
                    np.float32(st.avg), np.float32(st.stddev))
    else:  # the HIP statistics kernel, EXACT mode (every field bit-exact)
        import torch

        from nvidia_resiliency_ext.straggler import ops

        def stats_fn(ns, cap=8192):
            t = torch.from_numpy(np.ascontiguousarray(ns, np.uint32).view(np.int32)).cuda()
            g = ops.segment_stats_strided(t, 1, t.numel(), 0, t.numel(), cap=cap,
                                          mode=ops.STATS_EXACT).cpu()
            return (int(g.num[0]), np.float32(g.min[0]), np.float32(g.max[0]),
                    np.float32(g.med[0]), np.float32(g.avg[0]), np.float32(g.std[0]))
    gen = lambda R, K, S, seed, strag: O.gen_matrix(R, K, S, seed=seed, straggler=strag)  # noqa
    from unittest.mock import patch

    import torch

    rg = straggler.reporting.ReportGenerator(sc["scores"], gather_on_rank0=sc["gather"],
                                             node_name=f"node{rank}")
    outs, digests, gathers = [], [], []
    Stat = straggler.Statistic
    for t in range(sc["reports"]):
        _, ker = SC.build_rank_inputs(sc, rank, t, gen, stats_fn, OR.section_summary_torch_semantics)
        digests.append(SC.summaries_digest({}, ker))
        secs = fx["section_summaries"][t][rank]
        sec = {n: {Stat[k]: (v if k == "NUM" else float.fromhex(v)) for k, v in s.items()}
               for n, s in secs.items()}
        kd = {n: {Stat[k]: v for k, v in s.items()} for n, s in ker.items()}
        with patch("torch.distributed.all_gather_object",
                   wraps=torch.distributed.all_gather_object) as m:
            rep = rg.generate_report(sec, kd)
            gathers.append(m.call_count)
        outs.append(SC.encode_report(rep))
    return dict(outs=outs, digests=digests, gathers=gathers,
                mapper=dict(kernel=rg.name_mapper.kernel_name_to_id,
                            section=rg.name_mapper.section_name_to_id))
