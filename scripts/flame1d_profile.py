"""BASELINE config 2 (1D flame, 880 cells) for a rocprofv3 kernel trace: where a latency-bound step goes."""
import os
import sys
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "deepflame-dev_amd"))
import bench  # noqa: E402

print(bench.flame1d_line(steps=int(sys.argv[1]) if len(sys.argv) > 1 else 50, warmup=10))
