"""tools/replay_kernels.py: the timed-region kernel table keeps only the kernels between a region's two marker
launches (setup kernels outside it never appear) and reports the window, overlap-merged busy share and per-step
figures -- on a synthetic rocprofv3 kernel-trace CSV."""
import csv
import importlib.util
import os


def _tool():
    path = os.path.join(os.path.dirname(__file__), "..", "tools", "replay_kernels.py")
    spec = importlib.util.spec_from_file_location("replay_kernels", path)
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    return mod


def _trace(tmp_path, rows):
    d = tmp_path / "rk"
    d.mkdir()
    with open(d / "run_kernel_trace.csv", "w", newline="", encoding="utf-8") as f:
        w = csv.writer(f)
        w.writerow(["Kernel_Name", "Start_Timestamp", "End_Timestamp"])
        for name, s, e in rows:
            w.writerow([name, s, e])
    return str(d)


def test_replay_table_keeps_only_the_timed_region(tmp_path):
    rk = _tool()
    M = "void svoc::svoc_bench_marker_kernel(int*, int)"
    rows = [("void setup_rng(int)", 0, 5000),                     # setup: before the first marker
            (M, 6000, 6010),                                       # region 1 opens at 6010
            ("void svoc::round_kernel<4>(svoc::FastParams)", 7000, 9000),
            ("void svoc::commit_kernel(int)", 8000, 9500),         # overlaps the round: merged busy time
            ("void svoc::round_kernel<4>(svoc::FastParams)", 10000, 12000),
            (M, 16010, 16020),                                     # region 1 closes at 16010
            ("void after_region(int)", 17000, 18000),              # after the region: excluded
            (M, 20000, 20010), ("void region2_kernel(int)", 21000, 22000), (M, 23000, 23010)]
    d = _trace(tmp_path, rows)
    out = rk.render(d, "synthetic", region=1, steps=2)
    assert "setup_rng" not in out and "after_region" not in out and "region2_kernel" not in out
    assert "| `svoc::round_kernel<4>` | 2 | 1 | 4.0 | 2.0 | 2.0 | 40.0 |" in out
    assert "| `svoc::commit_kernel` | 1 | 0.5 | 1.5 | 1.5 | 0.8 | 15.0 |" in out
    # window 10.0 us; busy = [7000, 9500] + [10000, 12000] = 4.5 us -> 45.0 %
    assert "10.0 us for 2 steps = 5.0 us/step" in out and "running 45.0 %" in out
    out2 = rk.render(d, "synthetic", region=2, steps=1)
    assert "region2_kernel" in out2 and "round_kernel" not in out2
