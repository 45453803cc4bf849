"""Summarise rocprofv3 CSV output (kernel trace + PMC passes of tools/profile.sh).

usage: python tools/pmc_summary.py gpurun_out/prof [profiles/<round>/<name>]
Writes <dest>/kernel_stats.csv (copied), <dest>/pmc_summary.json and, under the profiled run's
workload key, profiles/pmc_latest.json (read by bench.py for roofline.traffic).  The key is taken
from the profiled run's own JSON line (<src>/trace.log: roofline.pmc_key, bench.workload_key), so a
bench line only ever finds the counters of a pass that ran its own workload.
"""
import csv, glob, json, os, shutil, sys
from collections import defaultdict

args = sys.argv[1:]
src = args[0]
dest = args[1] if len(args) > 1 else None


def workload_key():
    """roofline.pmc_key of the last JSON line the traced run printed (None if absent)"""
    for log in ('trace.log', 'pmc_fetch.log'):
        try:
            with open(os.path.join(src, log)) as fh:
                lines = [ln for ln in fh if ln.startswith('{')]
        except OSError:
            continue
        for ln in reversed(lines):
            try:
                k = json.loads(ln).get('roofline', {}).get('pmc_key')
            except ValueError:
                continue
            if k:
                return k
    return None

def newest(pattern):
    """Per directory only the newest run's file: gpurun merges every call's output into the same
    local gpurun_out/, so older runs' CSVs (other process ids) sit beside the current ones."""
    best = {}
    for f in glob.glob(os.path.join(src, pattern), recursive=True):
        d = os.path.dirname(f)
        if d not in best or os.path.getmtime(f) > os.path.getmtime(best[d]):
            best[d] = f
    return sorted(best.values())


def rows(pattern):
    out = []
    for f in newest(pattern):
        with open(f) as fh:
            out.extend(csv.DictReader(fh))
    return out

def short(name):
    if 'smem_kernel' in name:
        return 'smem_kernel'
    for kern in ('glob_lane_kernel', 'glob_band_kernel', 'glob_wide_kernel', 'wv_kernel', 'gq_kernel', 'pc_kernel',
                 'pk_kernel', 'lane_kernel', 'mate_kernel'):
        if kern in name:
            for q in ('160', '128', '96', '80', '64', '48', '32', '16', '10', '8', '6', '4'):
                if f'ILi{q}E' in name or f'<{q},' in name or f'<{q}>' in name:
                    return f'{kern}<{q}>'
            return kern
    for k in ('wide_kernel', 'plan_kernel', 'Radix', 'radix', 'Onesweep', 'onesweep'):
        if k in name:
            return k
    return name[:60]

summary = {}
stats = rows('**/*kernel_stats.csv')
for r in stats:
    n = short(r.get('Name', ''))
    summary.setdefault(n, {})
    summary[n]['calls'] = int(r.get('Calls', 0))
    summary[n]['avg_ns'] = float(r.get('AverageNs', 0))
    summary[n]['total_ns'] = float(r.get('TotalDurationNs', 0))
    summary[n]['pct'] = float(r.get('Percentage', 0))
# PMC: counter_collection.csv has one row per dispatch and counter
acc = defaultdict(lambda: defaultdict(list))
for r in rows('**/*counter_collection.csv'):
    n = short(r.get('Kernel_Name', ''))
    acc[n][r['Counter_Name']].append(float(r['Counter_Value']))
for n, cs in acc.items():
    d = summary.setdefault(n, {})
    for c, v in cs.items():
        d[c + '_per_launch'] = sum(v) / len(v)
    if 'FETCH_SIZE' in cs or 'WRITE_SIZE' in cs:
        # gfx950: FETCH_SIZE reports 1/2 of the bytes of streaming and LDS-DMA reads
        # (MI355X_MICROARCH.md "HBM"; calibrated for this kernel's access pattern in
        # profiles/r01/fetch_calibration.json) -> x2.  WRITE_SIZE is exact.
        # smem_kernel reads random 64-B occurrence blocks (one 64-B request each, tallied at
        # 64 B): no streaming half-count, raw FETCH_SIZE (uncalibrated for that width)
        k = 1 if n == 'smem_kernel' else 2
        f = d.get('FETCH_SIZE_per_launch', 0.0) * 1024 * k
        wr = d.get('WRITE_SIZE_per_launch', 0.0) * 1024
        d['fetch_bytes_per_launch'] = f
        d['write_bytes_per_launch'] = wr
        d['hbm_bytes_per_launch'] = f + wr
        d['fetch_correction'] = ('FETCH_SIZE x2 (gfx950 half-count, calibrated)' if k == 2 else
                                 'FETCH_SIZE raw (64-B random requests; uncalibrated)')
print(json.dumps(summary, indent=1))
if dest:
    os.makedirs(dest, exist_ok=True)
    for f in newest('**/*kernel_stats.csv')[:1]:
        shutil.copy(f, os.path.join(dest, 'kernel_stats.csv'))
    with open(os.path.join(dest, 'pmc_summary.json'), 'w') as fh:
        json.dump(summary, fh, indent=1)
    # profiles/pmc_latest.json: one entry per workload key (this pass replaces its own workload's)
    key = workload_key()
    if key is None:
        print('no roofline.pmc_key in the traced run\'s output: profiles/pmc_latest.json not updated', file=sys.stderr)
        sys.exit(0)
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    latest = os.path.join(root, 'profiles', 'pmc_latest.json')
    merged = {}
    if os.path.exists(latest):
        with open(latest) as fh:
            merged = json.load(fh)
    merged[key] = {'source': os.path.relpath(os.path.join(dest, 'pmc_summary.json'), root),
                   'kernels': {k: v for k, v in summary.items() if 'hbm_bytes_per_launch' in v}}
    with open(latest, 'w') as fh:
        json.dump(merged, fh, indent=1)
    print(f'pmc_latest.json[{key}] <- {merged[key]["source"]}', file=sys.stderr)
