"""Where the SMEM kernel's time goes: mem_collect_intv on the GPU with its passes switched off
one by one (pass 2 = re-seeding: split_width 0; pass 3 = LAST-like seeds: max_mem_intv 0), on
the bench's seeding reference of the given size, text mode and blocks-only.
usage: python tools/smem_phase_probe.py REF_MB READS"""
import os, sys, time
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "bwa-mem2-arm_amd", "py"))
import numpy as np
import bench, bsw, hiprt

mb, n = int(sys.argv[1]), int(sys.argv[2])
L, cap = 151, 256
t = time.perf_counter()
ref = bench.seeding_reference(mb * 1_000_000)
reads, off, lens = bench.seeding_reads(ref, n, L, seed=11)
print(f"generated {mb} Mb + {n} reads in {time.perf_counter() - t:.1f} s", flush=True)
d_reads, d_off, d_len = (hiprt.DeviceBuffer.from_array(a) for a in (reads, off, lens))
d_mems = hiprt.DeviceBuffer(n * cap * 32)
d_cnt = hiprt.DeviceBuffer(n * 4)
for flags in (None, bsw.FMI_NO_TEXT):
    fmi = bsw.Fmi(ref, flags=flags)
    for name, kw in (("all passes", {}), ("pass 1 only", dict(split_width=0, max_mem_intv=0)),
                     ("passes 1+2", dict(max_mem_intv=0)), ("passes 1+3", dict(split_width=0))):
        o = bsw.mem_opt(**kw)
        ms = []
        for _ in range(3):
            rc = fmi.collect_intv_device(d_reads.ptr, d_off.ptr, d_len.ptr, n, L, d_mems.ptr, cap, d_cnt.ptr, opt=o)
            assert rc == 0, rc
            ms.append(fmi.last_kernel_ms())
        cnt = d_cnt.download(np.zeros(n, np.int32))
        print(f"{'text' if flags is None else 'blocks'} {name:12s}: kernel {min(ms):8.2f} ms, "
              f"{cnt.mean():.2f} intervals/read", flush=True)
    fmi.close()
