"""The Scheduler's tie rule orders partitions by java.util.HashMap<String, …> iteration (JDK 8) over the
String.valueOf texts of the partition keys (Double / Float.toString for floating-point keys). Both are
restated twice, independently: the oracle's oracle/jhashmap.h and the product's host-side
siddhi_amd/csrc/sh_jmap.h. This CPU test drives both with the same random computeIfAbsent /
iterator-remove sequences (heavy String.hashCode collisions: tree bins, splits, untreeify) and requires
identical iteration orders at every step (tests/native/jmap_diff.cpp). The Java behaviour itself is
pinned by the hand-traced KAT `partition_tie_hashmap_order` (head insertion, bin order)."""
import os
import subprocess

HERE = os.path.dirname(os.path.abspath(__file__))


def test_two_restatements_of_java_hashmap_order_agree(tmp_path):
    exe = str(tmp_path / "jmap_diff")
    subprocess.run(["g++", "-O2", "-std=c++17", "-o", exe, os.path.join(HERE, "native", "jmap_diff.cpp")],
                   check=True)
    r = subprocess.run([exe, "40"], capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stdout + r.stderr
    assert r.stdout.startswith("ok"), r.stdout


# Double.toString / Float.toString (JDK 8 javadoc; the values below are the ones Java prints — the
# javadoc's own Double.MIN_VALUE "4.9E-324", Float.MAX_VALUE "3.4028235E38", Float.MIN_VALUE "1.4E-45")
JAVA_TEXT = [(1.0, "1.0"), (100.0, "100.0"), (1e7, "1.0E7"), (9999999.0, "9999999.0"), (0.001, "0.001"),
             (1e-4, "1.0E-4"), (-0.0, "-0.0"), (0.0, "0.0"), (float("nan"), "NaN"), (float("inf"), "Infinity"),
             (-float("inf"), "-Infinity"), (5e-324, "4.9E-324"), (1.7976931348623157e308, "1.7976931348623157E308"),
             (0.1, "0.1"), (1 / 3, "0.3333333333333333"), (123456.789, "123456.789"), (-2.5, "-2.5"), (1e21, "1.0E21"),
             (12345678.9, "1.23456789E7"), (2.2250738585072014e-308, "2.2250738585072014E-308"), (0.0015, "0.0015"),
             (0.1 + 0.2, "0.30000000000000004")]
JAVA_FLOAT_TEXT = [(1.1, "1.1"), (0.1, "0.1"), (3.4028234663852886e38, "3.4028235E38"), (1.401298464324817e-45, "1.4E-45"),
                   (16777216.0, "1.6777216E7"), (1 / 3, "0.33333334"), (100.0, "100.0")]


def test_java_fp_text_known_values():
    import numpy as np
    from oracle.oracle import fp_text
    for v, want in JAVA_TEXT:
        assert fp_text(v) == want, (v, want)
    for v, want in JAVA_FLOAT_TEXT:
        assert fp_text(float(np.float32(v)), True) == want, (v, want)


def test_two_restatements_of_java_fp_text_agree(tmp_path):
    exe = str(tmp_path / "fptext_diff")
    subprocess.run(["g++", "-O2", "-std=c++17", "-o", exe, os.path.join(HERE, "native", "fptext_diff.cpp")],
                   check=True)
    r = subprocess.run([exe, "400000"], capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stdout + r.stderr
    assert r.stdout.startswith("ok"), r.stdout
