"""Diagnostic: the first aggregation KAT on the GPU with SH_TRACE on."""
import faulthandler
import sys
sys.path.insert(0, ".")
faulthandler.dump_traceback_later(40, exit=True)
from siddhi_amd import runtime  # noqa: E402
from tests import kat_runner  # noqa: E402
case = [c for c in kat_runner.load_cases() if c.get("kind") == "aggregation"][0]
print("case", case["name"], flush=True)
schema, spec, dic, a = kat_runner.run_aggregation(case, runtime.GpuAggregation)
print("pushed", flush=True)
