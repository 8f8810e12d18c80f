"""Diagnostic: run one GPU query through the library, then report the HIP runtime's pending error on
this thread (hipPeekAtLastError) before torch initialises its own HIP context."""
import ctypes as C
import sys

import numpy as np

sys.path.insert(0, ".")
from siddhi_amd import abi, runtime  # noqa: E402
from tests.parity import split_batches  # noqa: E402

hip = C.CDLL("libamdhip64.so")
hip.hipGetErrorName.restype = C.c_char_p


def peek(label):
    e = hip.hipPeekAtLastError()
    print(label, e, hip.hipGetErrorName(e).decode(), flush=True)


peek("start")
rng = np.random.default_rng(11)
n = 50_000
schema = abi.Schema.parse("a int, b string, x int, y long, f float, d double")
cols = [rng.integers(-3, 3, n).astype(np.int32), rng.integers(0, 7, n).astype(np.int32),
        rng.integers(-10**6, 10**6, n).astype(np.int32), rng.integers(-10**12, 10**12, n).astype(np.int64),
        (rng.standard_normal(n) * 100).astype(np.float32), rng.standard_normal(n) * 1e6]
ts = np.arange(n, dtype=np.int64)
spec = abi.QuerySpec(schema, "lengthBatch", 333, group_by=["a", "b"],
                     aggs=[("sum", "x"), ("sum", "y"), ("sum", "f"), ("avg", "x"), ("avg", "f"), ("min", "f"),
                           ("max", "y"), ("min", "d")], key_capacity=64)
g = runtime.GpuQuery(spec)
peek("after create")
for i, p in enumerate(split_batches(schema, ts, cols, [1000, 1001, 30_000], 7)):
    g.push_raw(p)
    peek(f"after push {i}")
g.close()
peek("after close")
import torch  # noqa: E402
print("torch", torch.cuda.device_count(), torch.cuda.is_available(), flush=True)
x = torch.zeros(4).to(torch.device("cuda", 0))
print("torch tensor ok", x.sum().item(), flush=True)
