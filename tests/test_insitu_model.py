"""tools/insitu_model.py (the in-situ resource model behind DESIGN.md §9d) on a hand-made trace:
two launches overlapping for half of their time; the model's time-weighted rates must equal the
closed-form values."""
import csv
import json
import subprocess
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent

COUNTER_COLS = ["Dispatch_Id", "Grid_Size", "Kernel_Name", "Counter_Name", "Counter_Value"]
TRACE_COLS = ["Kernel_Name", "Start_Timestamp", "End_Timestamp", "Grid_Size_X", "Grid_Size_Y", "Grid_Size_Z"]
BLUR = "void vo::k_blur_stream<13, 0, 4>(float const*)"
DESC = "void vo::k_desc<4>(vo::Pyramid const*)"


def _write(path, cols, rows):
    with open(path, "w", newline="") as f:
        w = csv.DictWriter(f, fieldnames=cols)
        w.writeheader()
        w.writerows(rows)


def test_insitu_model_rates(tmp_path):
    pmc = tmp_path / "pmc" / "p1"
    pmc.mkdir(parents=True)
    # per launch: blur 4 GB (FETCH 1 GB in KiB x2 + WRITE 2 GB in KiB), desc 1e9 VALU wave-instructions
    rows = []
    for d in (1, 2):
        rows += [{"Dispatch_Id": d, "Grid_Size": 6400, "Kernel_Name": BLUR, "Counter_Name": "FETCH_SIZE",
                  "Counter_Value": 1e9 / 1024},
                 {"Dispatch_Id": d, "Grid_Size": 6400, "Kernel_Name": BLUR, "Counter_Name": "WRITE_SIZE",
                  "Counter_Value": 2e9 / 1024}]
    rows.append({"Dispatch_Id": 3, "Grid_Size": 64, "Kernel_Name": DESC, "Counter_Name": "SQ_INSTS_VALU",
                 "Counter_Value": 1e9})
    _write(pmc / "p_counter_collection.csv", COUNTER_COLS, rows)
    ms = 1_000_000                                   # ns
    trace = [  # blur A [0, 4 ms) (fill, partly dropped), blur B [4, 8 ms), desc [6, 10 ms)
        {"Kernel_Name": BLUR, "Start_Timestamp": 0, "End_Timestamp": 4 * ms, "Grid_Size_X": 6400, "Grid_Size_Y": 1,
         "Grid_Size_Z": 1},
        {"Kernel_Name": BLUR, "Start_Timestamp": 4 * ms, "End_Timestamp": 8 * ms, "Grid_Size_X": 6400,
         "Grid_Size_Y": 1, "Grid_Size_Z": 1},
        {"Kernel_Name": DESC, "Start_Timestamp": 6 * ms, "End_Timestamp": 10 * ms, "Grid_Size_X": 64,
         "Grid_Size_Y": 1, "Grid_Size_Z": 1},
    ]
    _write(tmp_path / "trace.csv", TRACE_COLS, trace)
    out = tmp_path / "m.json"
    subprocess.run([sys.executable, str(ROOT / "tools" / "insitu_model.py"), str(tmp_path / "pmc"),
                    str(tmp_path / "trace.csv"), str(out)], check=True, capture_output=True)
    d = json.loads(out.read_text())
    # window = [2.5, 10] ms (first quarter dropped): blur at 1 TB/s (4 GB / 4 ms) over [2.5, 8)
    assert abs(d["window_ms"] - 7.5) < 1e-9
    assert abs(d["mean"]["hbm_TBs"] - 1.0 * 5.5 / 7.5) < 1e-9
    # desc: 1e9 wave-instructions over 4 ms, 2 cycles each, 1024 SIMDs at 2.4 GHz
    valu = 1e9 * 2 / 4e-3 / (1024 * 2.4e9)
    assert abs(d["mean"]["valu_util"] - valu * 4 / 7.5) < 1e-9
    ts = d["time_share"]
    assert abs(ts["both_streams"] - 2 / 7.5) < 1e-9 and abs(ts["scale_only"] - 3.5 / 7.5) < 1e-9
    assert abs(ts["feature_only"] - 2 / 7.5) < 1e-9 and ts["idle"] == 0
    assert abs(d["below_3TBs"]["time_share"] - 1.0) < 1e-9      # 1 TB/s everywhere
