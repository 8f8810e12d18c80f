"""CPU-side checks of the drop-in boundary: the C-ABI library loads, exports every symbol the header
declares, and the ctypes structs match the C layout. No compute calls (no GPU here)."""
import ctypes as C
import os
import re
import subprocess

import pytest

from siddhi_amd import abi

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HDR = os.path.join(ROOT, "include", "siddhi_hip.h")
LIB = os.path.join(ROOT, "siddhi_amd", "libsiddhi_hip.so")


def header_functions():
    txt = open(HDR).read()
    return sorted(set(re.findall(r"^\s*(?:int|const char\*|int32_t)\s+(sh_\w+)\s*\(", txt, re.M)))


def test_header_declares_expected_symbols():
    assert header_functions() == sorted(abi.ABI_SYMBOLS)


@pytest.mark.skipif(not os.path.exists(LIB), reason="library not built")
def test_library_exports_every_header_symbol():
    out = subprocess.run(["nm", "-D", "--defined-only", LIB], capture_output=True, text=True, check=True).stdout
    exported = set(l.split()[-1] for l in out.splitlines() if l.strip())
    missing = [s for s in header_functions() if s not in exported]
    assert not missing, missing
    L = C.CDLL(LIB)
    L.sh_abi_version.restype = C.c_int32
    assert L.sh_abi_version() == 16


def test_struct_layout_matches_c(tmp_path):
    src = tmp_path / "sz.c"
    src.write_text('#include <stdio.h>\n#include <stddef.h>\n#include "siddhi_hip.h"\n'
                   'int main(void){printf("%zu %zu %zu %zu %zu %zu %zu %zu\\n", sizeof(sh_filter_op), sizeof(sh_query_desc),'
                   ' sizeof(sh_aggregation_desc), sizeof(sh_batch), sizeof(sh_out), sizeof(sh_stats),'
                   ' offsetof(sh_query_desc, key_capacity), offsetof(sh_out, nulls));'
                   'printf("%zu %zu\\n", sizeof(sh_slice_summary), sizeof(sh_bound));return 0;}\n')
    exe = tmp_path / "sz"
    subprocess.run(["gcc", "-I", os.path.join(ROOT, "include"), str(src), "-o", str(exe)], check=True)
    got = list(map(int, subprocess.run([str(exe)], capture_output=True, text=True, check=True).stdout.split()))
    want = [C.sizeof(abi.FilterOp), C.sizeof(abi.QueryDesc), C.sizeof(abi.AggregationDesc), C.sizeof(abi.Batch),
            C.sizeof(abi.Out), C.sizeof(abi.Stats), abi.QueryDesc.key_capacity.offset, abi.Out.nulls.offset,
            C.sizeof(abi.SliceSummary), C.sizeof(abi.Bound)]
    assert got == want


def test_product_path_refuses_without_gpu():
    """No HIP device in this container: the product library must fail loudly, never fall back."""
    if not os.path.exists(LIB):
        pytest.skip("library not built")
    import torch
    if torch.cuda.is_available():
        pytest.skip("GPU present")
    from siddhi_amd import runtime
    with pytest.raises(runtime.SiddhiError):
        runtime.Context(0)
