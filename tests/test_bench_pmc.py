"""bench.py's in-run PMC evidence (pmc_live) on CPU: the rocprofv3 passes are replaced by a stub that
writes the CSV files rocprofv3 writes, so the parsing, the gfx950 FETCH_SIZE correction, the per-launch
medians, the instruction pricing and the fallbacks are checked without a GPU."""
import argparse
import csv
import os
import shutil
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import bench  # noqa: E402

KERNEL = "void enf::flow_hj_kernel<32, 8, 2, 1, 4, 0, 1, 0, false>(enf::HJArgs)"
COUNTERS = {"FETCH_SIZE": 1_268_750.0, "SQ_WAVES": 40960.0, "WRITE_SIZE": 1_015_625.0, "SQ_WAVE_CYCLES": 4.0e9,
            "SQ_WAIT_INST_ANY": 1.9e9, "SQ_INSTS_VALU": 3.4448e8, "GRBM_GUI_ACTIVE": 1.12e7,
            "SQ_INSTS_VALU_TRANS_F32": 4.25e7, "SQ_INSTS_LDS": 1.42e7}
DUR_NS = [760_000, 740_000, 750_000]  # three profiled launches per pass: median 750 us


def _args():
    return argparse.Namespace(pairs=4, dtype="f32", pattern=None)


def _fake_runner(fail_pass=None, other_kernel=False):
    calls = []

    def run(cmd, timeout_s, log):
        calls.append(cmd)
        d = cmd[cmd.index("-d") + 1]
        os.makedirs(d, exist_ok=True)
        name = "void enf::some_other_kernel()" if other_kernel else KERNEL
        if "--stats" in cmd:
            with open(os.path.join(d, "run_kernel_stats.csv"), "w", newline="") as f:
                w = csv.writer(f)
                w.writerow(["Name", "Calls", "TotalDurationNs", "AverageNs", "Percentage", "MinNs", "MaxNs"])
                w.writerow([name, 23, 23 * 770000, 770000.0, 99.0, 668000, 882000])
            return 0
        if fail_pass is not None and d.endswith(f"p{fail_pass}"):
            return None  # timed out
        grp = cmd[cmd.index("--pmc") + 1:cmd.index("--output-format")]
        with open(os.path.join(d, "run_counter_collection.csv"), "w", newline="") as f:
            w = csv.writer(f)
            w.writerow(["Dispatch_Id", "Kernel_Name", "Counter_Name", "Counter_Value"])
            for disp in range(3):
                for c in grp:
                    # each counter split over two rows of one dispatch (per-XCD / per-SE instances are summed)
                    w.writerow([disp, name, c, COUNTERS[c] / 2])
                    w.writerow([disp, name, c, COUNTERS[c] / 2])
        with open(os.path.join(d, "run_kernel_trace.csv"), "w", newline="") as f:
            w = csv.writer(f)
            w.writerow(["Dispatch_Id", "Kernel_Name", "Start_Timestamp", "End_Timestamp"])
            for disp, dur in enumerate(DUR_NS):
                w.writerow([disp, name, 1000, 1000 + dur])
        return 0

    return run, calls


@pytest.fixture
def rocprof_present(monkeypatch):
    monkeypatch.setattr(shutil, "which", lambda name: "/opt/rocm/bin/rocprofv3")
    for k in list(os.environ):
        if k.startswith("ROCPROF"):
            monkeypatch.delenv(k)
    monkeypatch.setenv("LD_PRELOAD", "")


def test_pmc_live_summary(monkeypatch, rocprof_present, tmp_path):
    monkeypatch.setenv("TMPDIR", str(tmp_path))
    run, calls = _fake_runner()
    monkeypatch.setattr(bench, "_run_group", run)
    traffic, valu, stats = bench.pmc_live(32, 10_000_000, _args())
    # FETCH_SIZE (KiB) doubled per the gfx950 correction, plus WRITE_SIZE (KiB)
    assert traffic["bytes_per_launch"] == COUNTERS["FETCH_SIZE"] * 1024 * 2 + COUNTERS["WRITE_SIZE"] * 1024
    assert "this run" in traffic["source"]
    assert valu["insts_per_launch"] == COUNTERS["SQ_INSTS_VALU"]
    assert valu["insts_per_element_pair"] == pytest.approx(COUNTERS["SQ_INSTS_VALU"] / (1e7 * 32 * 4 / 64))
    clk = COUNTERS["GRBM_GUI_ACTIVE"] / 8 / 750_000
    assert valu["pmc_effective_clock_ghz"] == pytest.approx(clk)
    trans = COUNTERS["SQ_INSTS_VALU_TRANS_F32"]
    floor = (2.0 * (COUNTERS["SQ_INSTS_VALU"] - trans) + 7.5 * trans) / 1024
    assert valu["issue_floor_frac"] == pytest.approx(floor / (clk * 750_000))
    assert valu["wait_inst_any_frac"] == pytest.approx(COUNTERS["SQ_WAIT_INST_ANY"] / COUNTERS["SQ_WAVE_CYCLES"])
    assert stats["average_ms"] == pytest.approx(0.77) and stats["calls"] == 23
    # one pass per counter group plus the kernel-stats pass; every child is this bench with --no-pmc
    assert len(calls) == len(bench.PMC_PASSES) + 1
    for cmd in calls:
        i = cmd.index("--")
        assert cmd[0].endswith("rocprofv3") and cmd[i + 1] == sys.executable and "--no-pmc" in cmd[i:]
        assert "--pmc" not in cmd or not any(x in cmd for x in ("--sys-trace", "--hip-trace", "-s", "-r"))
    assert os.listdir(tmp_path) == []  # scratch directory removed


@pytest.mark.parametrize("kind", ["timeout", "no_kernel"])
def test_pmc_live_falls_back(monkeypatch, rocprof_present, tmp_path, kind):
    monkeypatch.setenv("TMPDIR", str(tmp_path))
    run, _ = _fake_runner(fail_pass=1) if kind == "timeout" else _fake_runner(other_kernel=True)
    monkeypatch.setattr(bench, "_run_group", run)
    assert bench.pmc_live(32, 10_000_000, _args()) is None
    assert os.listdir(tmp_path) == []


def test_pmc_live_never_nests(monkeypatch, rocprof_present):
    monkeypatch.setenv("ROCPROF_COUNTERS", "x")
    monkeypatch.setattr(bench, "_run_group", lambda *a: pytest.fail("a profiler pass started under a profiler"))
    assert bench.pmc_live(32, 10_000_000, _args()) is None


def test_cgroup_quota_parsing(monkeypatch, tmp_path):
    real_open = open

    def fake_open(path, *a, **k):
        if path == "/sys/fs/cgroup/cpu.max":
            p = tmp_path / "cpu.max"
            p.write_text(fake_open.text)
            return real_open(p, *a, **k)
        return real_open(path, *a, **k)

    monkeypatch.setattr("builtins.open", fake_open)
    fake_open.text = "1600000 100000\n"
    assert bench.cgroup_cpu_quota() == 16
    fake_open.text = "150000 100000\n"
    assert bench.cgroup_cpu_quota() == 2
    fake_open.text = "max 100000\n"
    assert bench.cgroup_cpu_quota() is None


def test_pmc_live_time_budget(monkeypatch, rocprof_present, tmp_path):
    """An exhausted budget starts no further pass (each pass is also killed at what is left of it)."""
    monkeypatch.setenv("TMPDIR", str(tmp_path))
    monkeypatch.setattr(bench, "PMC_BUDGET_S", 0.0)
    monkeypatch.setattr(bench, "_run_group", lambda *a: pytest.fail("a pass started past the budget"))
    assert bench.pmc_live(32, 10_000_000, _args()) is None
    seen = []
    monkeypatch.setattr(bench, "PMC_BUDGET_S", 1000.0)
    run, _ = _fake_runner()
    monkeypatch.setattr(bench, "_run_group", lambda cmd, t, log: (seen.append(t), run(cmd, t, log))[1])
    assert bench.pmc_live(32, 10_000_000, _args()) is not None
    assert seen and all(0 < t <= 90.0 for t in seen)


def test_kernel_match_tells_the_fp64_programs_apart():
    """The fp64 forward and inverse programs are one template, flow_hj64_kernel<D, U, LM, PAD, OCC, INV> (round 4):
    the in-run profiler passes of an --inverse --dtype f64 line must follow the INV = true launches only (the
    line's untimed forward pass runs the forward one), and the forward line the INV = false ones."""
    import types

    import bench

    fwd = "void enf::flow_hj64_kernel<32, 1, 1, false, 1, false>(enf::HJ64Args)"
    inv = "void enf::flow_hj64_kernel<32, 1, 1, false, 1, true>(enf::HJ64Args)"
    pad_inv = "void enf::flow_hj64_kernel<128, 1, 2, true, 1, true>(enf::HJ64Args)"
    a = types.SimpleNamespace(dtype="f64", inverse=True)
    assert bench.kernel_match(a, inv) and bench.kernel_match(a, pad_inv) and not bench.kernel_match(a, fwd)
    a = types.SimpleNamespace(dtype="f64", inverse=False)
    assert bench.kernel_match(a, fwd) and not bench.kernel_match(a, inv)
    a = types.SimpleNamespace(dtype="f32", inverse=False)
    assert bench.kernel_match(a, "void enf::flow_hj_kernel<32, 8, 2, 1, 4, 0, 1, false>(enf::HJArgs)")
    assert not bench.kernel_match(a, fwd)
    a = types.SimpleNamespace(dtype="f32", inverse=True)
    assert bench.kernel_match(a, "void enf::flow_hji_kernel<32, 8, 2, 1, false>(enf::HJArgs)")
    assert not bench.kernel_match(a, "void enf::flow_hj_kernel<32, 8, 2, 1, 4, 0, 1, false>(enf::HJArgs)")
