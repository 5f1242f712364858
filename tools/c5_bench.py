"""C5 tracker leg alone (bench.tracker_leg: detect + LK + associate per frame), for rocprofv3."""
import json, os, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench
print(json.dumps(bench.tracker_leg(0, 50, False)))
