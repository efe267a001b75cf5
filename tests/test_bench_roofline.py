"""CPU: bench.py's roofline fields reproduce from the committed PMC summaries (profiles/rNN_*_pmc.json):
the Mode X headline roofline is the VALU -- useful lane-op slots = pipe-weighted
VALU instructions x 64 x lane utilisation, against 1,024 SIMDs x 32 lanes x 2.4 GHz -- so its frac equals
valu_pipe_frac x valu_lane_util at the same kernel time; the binding resource is named."""
import json
import os
import sys

import pytest

import oracle_util as U

sys.path.insert(0, U.ROOT)
import bench  # noqa: E402


@pytest.mark.parametrize("workload,kernel", [("C3", "k_seg"), ("C2", "k_seg"), ("C4", "k_mode_x"), ("C5", "k_mode_x")])
def test_valu_roofline_reproduces_from_counters(workload, kernel):
    got = bench.pmc_summary(workload, kernel)
    assert got is not None, f"no committed PMC summary for {workload}"
    src, d = got
    c = d["counters_per_launch"]
    kern_ms = d["avg_launch_ns"] / 1e6
    ceil = bench.counter_ceilings(workload, kern_ms, kernel)
    f64 = sum(c[k] for k in ("SQ_INSTS_VALU_ADD_F64", "SQ_INSTS_VALU_MUL_F64", "SQ_INSTS_VALU_FMA_F64",
                             "SQ_INSTS_VALU_TRANS_F64"))
    slots = ((c["SQ_INSTS_VALU"] - f64) + 2.0 * f64) * 64.0
    assert ceil["valu_lane_slots"] == int(slots)
    lu = c["SQ_THREAD_CYCLES_VALU"] / (64.0 * c["SQ_ACTIVE_INST_VALU"])
    achieved = slots * lu / (kern_ms * 1e-3) / 1e12
    frac = achieved / bench.VALU_LANE_PEAK_TOPS
    # at the PMC run's own kernel time the frac is the pipe's busy share x its lane utilisation, except
    # for the clock: GRBM_GUI_ACTIVE / 8 cycles against kernel time x 2.4 GHz
    cycles = c["GRBM_GUI_ACTIVE"] / 8.0
    pipe = ((c["SQ_INSTS_VALU"] - f64) * 2.0 + f64 * 4.0) / (1024 * cycles)
    clock_ratio = cycles / (kern_ms * 1e-3 * 2.4e9)
    assert abs(frac - pipe * lu * clock_ratio) <= 1e-6 * max(1.0, frac)
    assert ceil["binding"] in ("latency", "valu", "hbm")
    assert 0.0 < frac < 1.0


def test_committed_c3_bench_line_carries_valu_roofline():
    p = os.path.join(U.ROOT, "profiles", "r06_bench", "C3.json")
    if not os.path.exists(p):
        pytest.skip("no round-6 C3 bench line committed")
    d = json.loads(open(p).read().strip().splitlines()[-1])
    r = d["roofline"]
    assert r["bound"] == "valu" and r["unit"] == "Tlane-op/s"
    assert abs(r["frac"] - r["achieved"] / r["peak"]) < 1e-4
    assert "hbm_alg_frac" in r and "hbm_counter_frac" in r
    assert d["cpu_baseline"]["cores_1t"] == 1 and d["cpu_baseline"]["value_1t"] > 0
    assert "bit-identical" in d["cpu_baseline"]["gpu_rows_check"]
