"""Diagnostic: one parity test through the library, then torch's first device tensor."""
import sys
sys.path.insert(0, ".")
from siddhi_amd import runtime  # noqa: E402
from tests import test_gpu_parity as t  # noqa: E402
t.test_lengthbatch_types_and_two_keys(runtime)
print("test ok", flush=True)
import torch  # noqa: E402
x = torch.zeros(4).to(torch.device("cuda", 0))
print("torch tensor ok", x.sum().item(), flush=True)
