"""Group-path statistics of pc_kernel on the C2 batch (experiment; GPU box):
   BSW_HIP_LIB=bwa-mem2-arm_amd/lib/libbsw_hip_stats.so python tools/pc_stats.py
Prints rows, groups entered / FAST / masked-R / masked-L, lastpos scans, per wave and per row."""
import ctypes
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "bwa-mem2-arm_amd", "py"))
import numpy as np  # noqa: E402
import hiprt  # noqa: E402
import bsw  # noqa: E402

pairs, ref, qer = bsw.synth_batch(int(os.environ.get("PAIRS", "1000000")))
d = [hiprt.DeviceBuffer.from_array(a) for a in (pairs, ref, qer)]
eng = bsw.Engine()
L = bsw.hip_lib()
L.bsw_pc_stats.argtypes = [ctypes.c_void_p, ctypes.c_int]
st = (ctypes.c_ulonglong * 8)()
eng.get_scores_device(d[0].ptr, d[1].ptr, d[2].ptr, len(pairs), 100, 16)
L.bsw_pc_stats(st, 1)
eng.get_scores_device(d[0].ptr, d[1].ptr, d[2].ptr, len(pairs), 100, 16)
L.bsw_pc_stats(st, 0)
rows, ent, fast, mr, ml, lp, waves, ue = (int(st[k]) for k in range(8))
print(f"waves {waves} rows {rows} ({rows / waves:.1f}/wave)  groups entered {ent} ({ent / rows:.2f}/row)")
print(f"FAST {fast / ent:.3f}  masked-R {mr / ent:.3f}  masked-L {ml / ent:.3f}  lastpos rows {lp / rows:.3f}")
print(f"uniform-end rows {ue / rows:.3f} (every live lane of the wave at the same band end)")
print(f"kernel_ms {eng.last_stats().kernel_ms:.3f}")
