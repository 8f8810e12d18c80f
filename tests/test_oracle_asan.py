"""The CPU restatement under AddressSanitizer + UndefinedBehaviorSanitizer (SURVEY.md §5's sanitizer
build; host code only): oracle/asan_driver.cpp drives every query shape the oracle restates — batch,
sliding and external-time windows with current / all / expired output, stream.current.event,
partitions, the five rate limiters and the sec...year aggregation with retrievals — on seeded streams.
Any sanitizer report aborts the driver; a failed call exits non-zero."""
import os
import subprocess

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_oracle_under_asan_and_ubsan():
    odir = os.path.join(ROOT, "oracle")
    subprocess.run(["make", "-s", "-C", odir, "asan_driver"], check=True, timeout=600)
    env = dict(os.environ, ASAN_OPTIONS="detect_leaks=1:abort_on_error=1",
               UBSAN_OPTIONS="halt_on_error=1:print_stacktrace=1")
    r = subprocess.run([os.path.join(odir, "asan_driver")], env=env, capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, r.stderr[-4000:]
    assert "aggregation sec..year" in r.stdout and "ERROR" not in r.stderr
