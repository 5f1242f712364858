"""Runs one bench.py leg alone and prints its JSON: python tools/leg.py live_path [cpu]."""
import json, os, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench
name = sys.argv[1]
cpu = len(sys.argv) > 2 and sys.argv[2] == "cpu"
fn = getattr(bench, name + "_leg")
out = fn(0, cpu) if name not in ("tracker",) else fn(0, 20, cpu)
print(json.dumps(out, indent=1))
