"""Time the reference's sequential loops on THIS host (the speedup
denominator of BASELINE.json's metric) and write profiles/host_seq_times.json."""
import json
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))
import bench  # noqa: E402

res = bench.measure_host_seq(2048)
(ROOT / "profiles").mkdir(exist_ok=True)
(ROOT / "profiles" / "host_seq_times.json").write_text(json.dumps(res, indent=1) + "\n")
print(json.dumps(res))
