"""The CPU baseline (oracle/cport/bgmres.c, C/OpenMP restatement of the reference Block GMRES
+ ICGS) on the bench workload (Laplace3D 256^3, k = 8, Num Blocks 25, tol 0) at 1 thread and
at the box's thread share, on the same sample of block iterations, one subprocess per thread
count (OMP_NUM_THREADS is read when the OpenMP runtime starts).  Not part of the tests.
  python tools/cpu_baseline_threads.py [iters] [threads...]"""
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
iters = int(sys.argv[1]) if len(sys.argv) > 1 else 5
threads = [int(t) for t in sys.argv[2:]] or [1, 16]
code = ("import sys, json; sys.path.insert(0, %r); import bench; "
        "print(json.dumps(bench.cpu_baseline(8, 25, 256, %d)))" % (ROOT, iters))
out = {}
for t in threads:
    env = dict(os.environ, OMP_NUM_THREADS=str(t))
    r = subprocess.run([sys.executable, "-c", code], env=env, capture_output=True, text=True, check=True)
    out[str(t)] = json.loads(r.stdout.strip().splitlines()[-1])
print(json.dumps(out))
