"""The Scheduler's tie rule orders partitions by java.util.HashMap<String, …> iteration (JDK 8). It is
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
