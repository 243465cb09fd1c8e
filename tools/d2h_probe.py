"""Copy of the gathered landmark map (float32 [L, 3], L = 3.49 M rows at KITTI-00: 42 MB) from HBM
to host memory on rank 0, the last step of kitti.finish_shard: pageable .cpu() vs a freshly pinned
tensor vs a pinned tensor re-used from torch's caching host allocator.  Prints ms per copy."""
import sys
import time

import torch


def main(rows: int = 3_494_012, reps: int = 5):
    d = torch.randn((rows, 3), device="cuda:0")
    torch.cuda.synchronize()

    def best(fn):
        ts = []
        for _ in range(reps):
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            r = fn()
            torch.cuda.synchronize()
            ts.append((time.perf_counter() - t0) * 1e3)
            del r
        return round(min(ts), 3), round(sorted(ts)[len(ts) // 2], 3)

    out = {"rows": rows, "mb": rows * 12 / 1e6}
    out["pageable_cpu"] = best(lambda: d.cpu().numpy())

    def fresh_pinned():
        h = torch.empty(d.shape, dtype=d.dtype, pin_memory=True)
        h.copy_(d)
        return h.numpy()
    out["pinned_alloc_copy"] = best(fresh_pinned)      # reps > 1 re-use the cached block
    h = torch.empty(d.shape, dtype=d.dtype, pin_memory=True)
    out["pinned_copy_only"] = best(lambda: h.copy_(d))
    out["pinned_copy_then_numpy_copy"] = best(lambda: h.copy_(d).numpy().copy())
    print(out, flush=True)


if __name__ == "__main__":
    main(*[int(a) for a in sys.argv[1:]])
