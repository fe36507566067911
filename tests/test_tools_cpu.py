"""Measurement tooling on the CPU: bench.py's warm-up call plan and tools/pmc_summary.py's choice of the
timed dispatches in a counter pass (the per-launch traffic the bench line reports comes from it)."""
import csv
import json
import os
import subprocess
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)

from bench import warmup_calls  # noqa: E402


def test_warmup_calls():
    assert warmup_calls(0, 120) == []
    assert warmup_calls(1, 120) == [1]
    assert warmup_calls(5, 120) == [2, 3]                  # the driver's shape: two warm-up calls
    assert warmup_calls(120, 120) == [60, 60]              # the default bench
    assert warmup_calls(300, 120) == [120, 120, 60]
    assert all(sum(warmup_calls(w, 120)) == w for w in range(0, 400, 7))


def _counter_csv(path, counter, values, kname="void hmcx::k_sghmc_p2<double, 10, 1>(hmcx::Q2Args)"):
    os.makedirs(path, exist_ok=True)
    with open(os.path.join(path, "run_counter_collection.csv"), "w", newline="") as fh:
        w = csv.DictWriter(fh, fieldnames=["Dispatch_Id", "Kernel_Name", "Counter_Name", "Counter_Value"])
        w.writeheader()
        for i, v in enumerate(values):
            for half in (0.5, 0.5):                          # two rows per dispatch (per-XCD style), summed
                w.writerow({"Dispatch_Id": 10 + i, "Kernel_Name": kname, "Counter_Name": counter,
                            "Counter_Value": v * half})
            w.writerow({"Dispatch_Id": 100 + i, "Kernel_Name": "other_kernel", "Counter_Name": counter,
                        "Counter_Value": 1e9})


def test_pmc_summary_picks_the_timed_dispatch(tmp_path):
    """bench.py --steps 20 --warmup 5: two warm-up launches, one timed, two diagnostics — the summary must
    use dispatch 2 (the round-4 closing run first read dispatch 1, a warm-up call)."""
    _counter_csv(tmp_path / "f", "FETCH_SIZE", [10.0, 20.0, 30.0, 40.0, 50.0])
    _counter_csv(tmp_path / "w", "WRITE_SIZE", [1.0, 2.0, 3.0, 4.0, 5.0])
    bj = tmp_path / "bench.json"
    bj.write_text(json.dumps({"warmup": 5, "steps": 20, "leapfrogs": 182.0, "roofline": {"calls": 1}}) + "\n")
    out = tmp_path / "pmc.json"
    r = subprocess.run([sys.executable, os.path.join(REPO, "tools", "pmc_summary.py"), str(tmp_path / "f"),
                        str(tmp_path / "w"), "k_sghmc_p2<double, 10", str(bj), str(out)],
                       capture_output=True, text=True, timeout=60)
    assert r.returncode == 0, r.stderr
    d = json.loads(out.read_text())
    assert d["fetch_size_kb_timed_mean"] == 30.0 and d["write_size_kb_timed_mean"] == 3.0
    assert d["traffic_bytes_per_launch"] == (2 * 30.0 + 3.0) * 1024.0
    assert d["leapfrogs_per_launch"] == 182.0


def test_hot_kernels_use_no_scratch():
    """The built library's hot kernels keep everything in registers: a kernel that spills to scratch runs
    several times slower (round 5: one k_wgrad edit spilled 2,264 VGPRs, 20.6 -> 175 us per config-5
    step) while staying correct, so no parity test would notice.  Reads the gfx950 code objects'
    metadata (tools/kernel_resources.py); skipped when libhmcx.so has not been built."""
    import re
    import pytest
    lib = os.path.join(REPO, "dropout_hamiltonian_montecarlo_amd", "lib", "libhmcx.so")
    if not os.path.exists(lib):
        pytest.skip("libhmcx.so not built")
    sys.path.insert(0, os.path.join(REPO, "tools"))
    import kernel_resources as kr
    ks = {}
    for co in kr.code_objects(kr.fatbin(lib)):
        for k in kr.kernels(co):
            ks[k["symbol"][:-3]] = k
    names = sorted(ks)
    # (the MLP GEMM kernels are not in this list: capped at 128 VGPRs so that four fused forwards are
    # co-resident, they spill a few registers — DESIGN §5.3)
    hot = re.compile(r"k_sghmc_p2<double, 10, 1>|k_wgrad<|k_wfwd_sm<|k_wfwd<|k_bfwd<|k_bgradw<|k_bgrad<|"
                     r"k_fwd<|k_grad<|k_binit<|k_wsoft<")
    checked, bad = 0, []
    for sym, dn in zip(names, kr.demangle(names)):
        if hot.search(dn):
            checked += 1
            if int(ks[sym].get("private_segment_fixed_size", 0)):
                bad.append((dn, ks[sym].get("private_segment_fixed_size")))
    assert checked >= 20, checked
    assert not bad, bad
