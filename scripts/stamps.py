"""Phase stamps of the C2 pipeline's kernels (diagnostic build, `make -C siddhi_amd/csrc stamps`).

Runs the default C2 workload through libsiddhi_hip_stamps.so, clears the stamp buffer, pushes one batch
and prints, per stamped kernel, the median / p90 cycles between consecutive stamp points of its
workgroups and the spread of workgroup start times. Usage: python scripts/stamps.py [kernel ids]"""
import ctypes as C
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
os.environ["SH_LIB"] = os.path.join(HERE, "..", "siddhi_amd", "libsiddhi_hip_stamps.so")
sys.path.insert(0, os.path.join(HERE, ".."))

import torch  # noqa: E402

from siddhi_amd import abi, runtime, synth  # noqa: E402

KERNELS = {0: "k_aggregate_own", 1: "k_ms_scatter", 2: "k_emit_rank", 3: "k_boundaries"}
NK, NB, NP = 4, 32768, 16


def main():
    dev = torch.device("cuda", 0)
    lib = C.CDLL(os.environ["SH_LIB"])
    lib.sh_debug_stamps.argtypes = [C.POINTER(C.c_ulonglong), C.c_longlong, C.c_int]
    ctx = runtime.Context(0)
    schema = abi.Schema.parse("k string, v double, ts long")
    spec = abi.QuerySpec(schema, "timeBatch", 1000, group_by=["k"],
                         aggs=[("count", None), ("min", "v"), ("max", "v"), ("avg", "v")], key_capacity=100_000)
    q = runtime.GpuQuery(spec, ctx)
    B = 1 << 25
    for i in range(3):
        ts, cols = synth.torch_keyed_stream(i * B, B, 0xC2, 100_000, 1000, dev)
        torch.cuda.synchronize()
        if i == 2:
            lib.sh_debug_stamps(None, 0, 1)
        q.push_device(B, ts.data_ptr(), [c.data_ptr() for c in cols], 1)
    torch.cuda.synchronize()
    buf = (C.c_ulonglong * (NK * NB * NP))()
    lib.sh_debug_stamps(buf, NK * NB * NP, 0)
    a = np.frombuffer(buf, dtype=np.uint64).reshape(NK, NB, NP).astype(np.int64)
    want = [int(x) for x in sys.argv[1:]] or list(KERNELS)
    for k in want:
        blk = a[k]
        used = blk[:, 0] > 0
        if not used.any():
            continue
        b = blk[used]
        npts = int((b > 0).sum(axis=1).max())
        print(f"{KERNELS[k]}: {used.sum()} workgroups, {npts} points")
        t0 = b[:, 0].min()
        print(f"  start spread: {(b[:, 0] - t0).max()} cycles; end {(b[:, npts - 1] - t0).max()} cycles")
        for p in range(1, npts):
            d = b[:, p] - b[:, p - 1]
            d = d[(b[:, p] > 0) & (b[:, p - 1] > 0)]
            print(f"  {p - 1}->{p}: median {np.median(d):8.0f}  p90 {np.percentile(d, 90):8.0f}  mean {d.mean():8.0f}")
        tot = b[:, npts - 1] - b[:, 0]
        print(f"  total: median {np.median(tot):8.0f}  p90 {np.percentile(tot, 90):8.0f}")
    q.close()


if __name__ == "__main__":
    main()
