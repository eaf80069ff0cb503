"""The agent's B = 1 call alone (bench.agent_call_gpu: /root/reference/agent.py:154,171-184, N = 15, dyn, fp64,
the reference's options) on n instances, for rocprofv3 counter passes on that launch shape.
Usage: python agent_probe.py [n]   (prints one JSON line: kernel / call p50, p90 and the status histogram)"""
import json
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, REPO)

import bench  # noqa: E402

if __name__ == "__main__":
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 20
    print(json.dumps(bench.agent_call_gpu(0, n=n)))
