"""Multi-process worlds for tests: spawn `ws` ranks on gloo (file store, 127.0.0.1 only),
run a module-level worker in each, return every rank's result.  Mirrors the reference's
tests/straggler/unit/_utils.py:121-178 pattern (torch.multiprocessing spawn + gloo)."""
import os
import sys
import tempfile
import traceback

import torch.multiprocessing as mp

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PATHS = [os.path.join(ROOT, "nvidia-resiliency-ext-x_amd"), os.path.join(ROOT, "oracle"),
         os.path.join(ROOT, "tests"), os.path.join(ROOT, "tests", "golden")]


def _entry(rank, ws, store, module, fn, kwargs, q):
    for p in PATHS:
        if p not in sys.path:
            sys.path.insert(0, p)
    try:
        import importlib

        import torch

        os.environ["RANK"] = str(rank)
        os.environ["WORLD_SIZE"] = str(ws)
        os.environ["LOCAL_RANK"] = "0"  # every rank shares the one test GPU
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        torch.distributed.init_process_group("gloo", init_method=f"file://{store}", rank=rank,
                                             world_size=ws)
        res = getattr(importlib.import_module(module), fn)(rank=rank, ws=ws, **kwargs)
        q.put((rank, "ok", res))
        torch.distributed.barrier()
        torch.distributed.destroy_process_group()
    except BaseException:  # report, do not hang the parent
        q.put((rank, "error", traceback.format_exc()))
        raise


def run_world(ws, module, fn, timeout=240, **kwargs):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    with tempfile.NamedTemporaryFile(delete=True) as tf:
        store = tf.name
    ps = [ctx.Process(target=_entry, args=(r, ws, store, module, fn, kwargs, q))
          for r in range(ws)]
    for p in ps:
        p.start()
    out = {}
    errors = []
    try:
        for _ in range(ws):
            rank, status, res = q.get(timeout=timeout)
            if status != "ok":
                errors.append(f"rank {rank}:\n{res}")
            out[rank] = res
    finally:
        for p in ps:
            p.join(timeout=30)
            if p.is_alive():
                p.kill()
    if errors:
        raise AssertionError("\n".join(errors))
    return out
