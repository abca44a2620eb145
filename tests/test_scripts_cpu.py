"""The measurement scripts on CPU: scripts/gpu.sh parses and lists its
tasks; the trace summarisers (trace_busy.py, kstats_tail.py) give the right
numbers on a small synthetic rocprofv3 kernel trace."""
import csv
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_gpu_sh_parses_and_lists_tasks():
    subprocess.check_call(["bash", "-n", os.path.join(ROOT, "scripts", "gpu.sh")])
    r = subprocess.run(["bash", os.path.join(ROOT, "scripts", "gpu.sh")], capture_output=True, text=True,
                       env=dict(os.environ, GRAFT_REPO_ROOT=ROOT))
    assert r.returncode == 2
    for task in ("round", "evidence", "ab", "kstats", "pmc", "pcie-trace", "route-trace", "seed-sweep",
                 "split-prof"):
        assert task in r.stdout, task


def _trace(path):
    # 4 batches of 100 us: k_prepare 0-20, k_table 20-80 (and an overlapping
    # k_part 30-50), idle 80-100
    rows = []
    for b in range(4):
        t = b * 100_000
        for name, s, e in (("rl::k_prepare(x)", 0, 20), ("rl::k_part(x)", 30, 50), ("rl::k_table(x)", 20, 80)):
            rows.append({"Kernel_Name": name, "Start_Timestamp": t + s * 1000, "End_Timestamp": t + e * 1000,
                         "Queue_Id": 1, "Grid_Size_X": 256, "Workgroup_Size_X": 256, "VGPR_Count": 32,
                         "Scratch_Size": 0})
    with open(path, "w", newline="") as f:
        w = csv.DictWriter(f, fieldnames=list(rows[0]))
        w.writeheader()
        w.writerows(rows)


def test_trace_busy_and_kstats_tail(tmp_path):
    p = str(tmp_path / "run_kernel_trace.csv")
    _trace(p)
    out = subprocess.check_output([sys.executable, os.path.join(ROOT, "scripts", "trace_busy.py"), p, "2", "0"],
                                  text=True)
    assert "100.0 us per batch" in out and "GPU busy 80.0 %" in out
    assert "k_table" in out and "60.0 us per batch" in out
    out = subprocess.check_output([sys.executable, os.path.join(ROOT, "scripts", "kstats_tail.py"), p, "2"],
                                  text=True)
    assert "rl::k_table" in out and "60" in out
