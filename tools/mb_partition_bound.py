"""Lower bound for a coarse-partition bucketing of configs[3]: the
partition pass must at least read and write every 8-B record once, and the bucketing pass after
it must read them again and write 4 B per record.  Times, on the configs[3] record volume
(16,384 x 47,482 records): a device copy of the records (read 8 + write 8 B / record) and a
read 8 + write 4 B / record pass (the keys half of the records, strided copy).  Prints JSON."""
import json

import torch

R, N = 16384, 47482
recs = torch.empty((R * N, 2), dtype=torch.int32, device="cuda")
recs.random_(0, 1 << 30)
dst = torch.empty_like(recs)
keys = torch.empty((R * N,), dtype=torch.int32, device="cuda")


def timed(fn, reps=10):
    fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / reps


copy_ms = timed(lambda: dst.copy_(recs))
keys_ms = timed(lambda: keys.copy_(recs[:, 1]))
nbytes = R * N * 8
print(json.dumps({
    "records": R * N,
    "copy_8r_8w_ms": round(copy_ms, 4), "copy_TBps": round(2 * nbytes / copy_ms / 1e9, 3),
    "keys_8r_4w_ms": round(keys_ms, 4), "keys_TBps": round(1.5 * nbytes / keys_ms / 1e9, 3),
    "partition_plus_bucket_lower_bound_ms": round(copy_ms + keys_ms, 4),
}), flush=True)
