import os
# kernel arms and knobs exist only in the tuning build (make -C zarr-python_amd tune)
os.environ.setdefault("ZARR_HIP_ALLOW_LIB_OVERRIDE", "1")
os.environ.setdefault("ZHIP_LIB", os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                                               "zarr-python_amd", "zarr_hip", "_lib", "libzarrhip_tune.so"))
import sys, os, json
sys.path.insert(0, "."); sys.path.insert(0, "zarr-python_amd")
import bench
from zarr_hip import _native as N
k = int(os.environ.get("K", "8"))
if k != 8:
    N.lib().zhip_set_tuning(3, k)
import torch
args = type("A", (), {"steps": 40, "tune": 0})()
r = bench.c1_plumbing(torch.device("cuda:0"), args)
print(json.dumps({"K": k, **{kk: r[kk] for kk in ("decoded_GiBps", "kernel_ms", "hbm_frac")}}))
