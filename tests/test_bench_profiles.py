"""bench.py's use of the committed rocprofv3 profiles (profiles/LATEST): the PMC figures it attaches
to the roofline and HBM fields come from the profile of the same workload (config and per-GPU proof
count) or are left out, and the committed profile holds what DESIGN.md cites (trace, PMC passes,
the default bench line with its roofline and cpu_baseline objects)."""
import json
import os

import pytest

import bench

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _latest():
    parts = open(os.path.join(ROOT, "profiles", "LATEST")).read().split()
    return parts[0], int(parts[1]), int(parts[2])


def _workload():
    """(AIR, input form) of the LATEST profile (a 3-field line: synthetic AIR, canonical words)."""
    parts = open(os.path.join(ROOT, "profiles", "LATEST")).read().split()
    return (parts[3] if len(parts) > 3 else "synthetic"), (parts[4] if len(parts) > 4 else "canonical")


@pytest.fixture(autouse=True)
def _latest_workload(monkeypatch):
    air, form = _workload()
    monkeypatch.setitem(bench.WORKLOAD, "air", air)
    monkeypatch.setitem(bench.WORKLOAD, "input_form", form)


def _profiled_lib(tag):
    import pytest
    f = os.path.join(ROOT, "profiles", tag, "LIB_SHA256")
    if not os.path.exists(f):
        pytest.skip(f"profiles/{tag} predates library hashing: no PMC figure is attached from it")
    return open(f).read().split()[0]


def test_latest_profile_is_keyed_by_workload_and_library(monkeypatch):
    tag, cfg, n = _latest()
    lib = _profiled_lib(tag)
    monkeypatch.setattr(bench, "lib_sha256", lambda path=None: lib)
    assert bench.latest_profile(cfg, n) == tag
    assert bench.latest_profile(cfg, n // 8) is None  # another per-GPU batch size
    assert bench.latest_profile(3 if cfg != 3 else 4, n) is None
    # another AIR or input form: another workload
    air, form = _workload()
    monkeypatch.setitem(bench.WORKLOAD, "air", "synthetic" if air != "synthetic" else "triton-size")
    assert bench.latest_profile(cfg, n) is None
    monkeypatch.setitem(bench.WORKLOAD, "air", air)
    monkeypatch.setitem(bench.WORKLOAD, "input_form", "canonical" if form != "canonical" else "montgomery")
    assert bench.latest_profile(cfg, n) is None
    monkeypatch.setitem(bench.WORKLOAD, "input_form", form)
    # counters of another binary are never attached
    monkeypatch.setattr(bench, "lib_sha256", lambda path=None: "0" * 64)
    assert bench.latest_profile(cfg, n) is None
    assert bench.pmc_traffic("k_mp_hash", cfg, n) == (None, None)
    assert bench.pmc_valu_per_step(cfg, n) == (None, None)


def test_fraction_guard():
    import pytest
    bench._assert_fracs({"a": {"frac": 0.4, "tip5_valu_frac": 0.2, "vs_regular_rate": 1.03}})
    with pytest.raises(AssertionError):
        bench._assert_fracs({"valu_issue": {"frac": 1.024}})


def test_latest_profile_files_and_pmc_figures(monkeypatch):
    tag, cfg, n = _latest()
    _profiled_lib(tag)
    d = os.path.join(ROOT, "profiles", tag)
    for f in ("SUMMARY.md", "bench_default.json", "bench_trace.json", "trace_kernel_stats.csv",
              "pmc_valu_counter_collection.csv", "pmc_fetch_counter_collection.csv",
              "pmc_write_counter_collection.csv", "LIB_SHA256"):
        assert os.path.exists(os.path.join(d, f)), f
    monkeypatch.setattr(bench, "lib_sha256", lambda path=None: _profiled_lib(tag))
    traffic, t_tag = bench.pmc_traffic("k_mp_hash", cfg, n)
    valu, v_tag = bench.pmc_valu_per_step(cfg, n)
    nbytes, b_tag = bench.pmc_bytes_per_step(cfg, n)
    assert t_tag == v_tag == b_tag == tag
    b = json.load(open(os.path.join(d, "bench_default.json")))
    rf = b["roofline"]
    # the level kernel moves about its algorithmic 80 B in + 40 B out per permutation
    assert 0.8 < traffic / (rf["perms_per_launch"] * 120) < 1.5
    assert valu > 1e9 and nbytes > 1e9
    assert b["config"]["workload"].startswith("BASELINE config 4") and b["n_gpus"] == 1
    assert rf["bound"] == "valu" and 0 < rf["frac"] < 1 and b["cpu_baseline"]["cores"] >= 1
    assert b["verdicts_correct"] is True
    # the default bench line of the profile was made with the profiled library
    assert b["config"]["lib_sha256"] == _profiled_lib(tag)[:16]


def test_summary_reproduces_the_bench_roofline():
    """SUMMARY.md's figures from the kernel traces agree with the bench's under the profiler: the
    reported (isolated-launch) roofline within 2%.  The in-flight side field is a looser check: with
    8 steps in flight (round 4) a launch's HIP start event is stamped while its dispatch still waits
    behind the other steps' kernels, so the bench's average runs above the trace's dispatch time
    (+14% in profiles/r04r; within 1% at round 3's 2 in flight)."""
    tag, _, _ = _latest()
    _profiled_lib(tag)
    text = open(os.path.join(ROOT, "profiles", tag, "SUMMARY.md")).read()
    line = next(x for x in text.splitlines() if x.startswith("roofline frac from the trace:"))
    frac_trace = float(line.split("T = ")[1].split(";")[0])
    frac_bench = float(line.rsplit("frac ", 1)[1])
    assert 0.97 < frac_trace / frac_bench < 1.25, (frac_trace, frac_bench)
    # the reported (isolated-launch) roofline: the trace of the one-at-a-time steps within 2%
    iso = [x for x in text.splitlines() if x.startswith("isolated roofline frac from the trace:")]
    if iso:  # (profiles from round 4 on)
        f_t = float(iso[0].split(": ")[1].split(";")[0])
        f_b = float(iso[0].rsplit("frac ", 1)[1])
        assert abs(f_t / f_b - 1) < 0.02, (f_t, f_b)


def test_inflight_defaults_and_queue_budget():
    """Steps in flight per per-GPU batch size (the driver's N = 1 / 2 / 4 / 8 shares of config 4
    and config 5's small batches) and the hardware queues bench.py provisions for them: every batch
    stream keeps its own queue, and no process asks for more than the 22 past which the device
    collapses (a rank of a multi-rank run also holds torch's and RCCL's streams: 9 in flight at
    512 proofs instead of 10)."""
    assert [bench.default_inflight(n) for n in (4096, 2048, 1024, 512, 64, 8)] == [8, 8, 8, 10, 20, 20]
    assert [bench.default_inflight(n, True) for n in (4096, 2048, 1024, 512, 64, 8)] == [8, 8, 8, 9, 18, 18]
    assert [bench.streams_for(n) for n in (4096, 512, 65, 64, 8)] == [2, 2, 2, 1, 1]
    for n in (4096, 2048, 1024, 512, 64, 8):
        for multi in (False, True):
            r = bench.default_inflight(n, multi)
            k = bench.streams_for(n)  # one stream per batch for the tiny ones
            q = bench.hw_queues_wanted(r, multi, k)
            streams = k * r + 1 + (2 if multi else 0)  # batch streams, the context's, torch + RCCL
            assert 8 <= q <= 22 and q >= streams, (n, multi, q, streams)
    assert bench.hw_queues_wanted(16, True) == 22
