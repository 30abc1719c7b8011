"""Rank workers for the kernel-hash sharded multi-GPU path (run inside tests/_mp.run_world)."""
import numpy as np


def oracle_shard_partials(rank, ws, R, K, S, cap):
    """CPU: each rank scores its hash shard of the kernel columns with the oracle; the
    [R][6] partials are all_gathered (gloo) and combined in shard order."""
    import torch

    import oracle as O
    from nvidia_resiliency_ext.straggler import synth

    ns = O.gen_matrix(R, K, S)
    st = O.matrix_stats(ns.reshape(-1), R * K, S, 0, S, cap)
    num, med, avg = (st[f].reshape(R, K) for f in ("num", "med", "avg"))
    ref = O.kernel_ref(num, med)  # shard-local in the real path: every GPU holds all ranks
    names = synth.kernel_names(K)
    mine = np.zeros(K, np.uint8)
    mine[synth.shard_kernels(names, ws, rank)] = 1
    part = torch.from_numpy(O.score_partials(num, med, avg, ref, col_in_shard=mine))
    gathered = torch.empty((ws * R, 6), dtype=torch.float64)
    torch.distributed.all_gather_into_tensor(gathered, part)
    gathered = gathered.view(ws, R, 6)
    tot = np.zeros((R, 6))
    for g in range(ws):  # fixed shard order
        tot = tot + gathered[g].numpy()
    rel = np.where(tot[:, 2] > 0, tot[:, 0] / np.where(tot[:, 1] == 0, 1, tot[:, 1]), np.nan)
    ind = np.where(tot[:, 5] > 0, tot[:, 3] / np.where(tot[:, 4] == 0, 1, tot[:, 4]), np.nan)
    return dict(rel=rel, ind=ind, owned=int(mine.sum()))


def gpu_sharded_report(rank, ws, R, K, S, cap, thr):
    """GPU (gloo, all ranks on one device): MatrixReporter over this rank's kernel shard."""
    import torch

    from nvidia_resiliency_ext.straggler import batch, synth

    names = synth.kernel_names(K)
    kidx = synth.shard_kernels(names, ws, rank)
    dev = torch.device("cuda:0")
    ns = synth.synth_matrix(R, len(kidx), S, K_global=K,
                            kmap=torch.from_numpy(kidx).to(dev), device=dev)
    rep = batch.MatrixReporter(R, len(kidx), cap=cap, thr_rel=thr, thr_ind=thr, device=dev)
    out = []
    for _ in range(2):  # second report exercises the persistent history
        r = rep.report(ns, S)
        out.append(dict(rel=r.gpu_relative, ind=r.gpu_individual, srel=r.stragglers_relative,
                        sind=r.stragglers_individual, err=r.err))
    return out
