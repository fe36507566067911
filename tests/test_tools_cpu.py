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
