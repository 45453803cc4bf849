"""pytest configuration: markers and import paths.

`-m "not gpu"`: oracle vs golden vectors / KATs / Python transcription, SSE4.1 baseline vs
oracle, C-ABI library loads and exports every declared symbol, synthetic generator,
multi-process (gloo) sharding -- all on CPU.
`-m gpu`: parity of the HIP path (called through the C ABI) against the CPU oracle.
"""

import os
import sys

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for sub in ("oracle", "tests", os.path.join("bwa-mem2-arm_amd", "py")):
    p = os.path.join(ROOT, sub)
    if p not in sys.path:
        sys.path.insert(0, p)



def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (gfx950) and the built HIP library")


def load_golden():
    """[(name, pairs, ref, qer, w, scoring), ...] from the committed fixtures: golden_v1.npz
    (manifest.json) and golden_v2.npz (manifest_v2.json)."""
    import json
    import bswgen
    out = []
    for mname, fname in (("manifest.json", "golden_v1.npz"), ("manifest_v2.json", "golden_v2.npz")):
        meta = json.load(open(os.path.join(ROOT, "tests", "golden", mname)))
        z = np.load(os.path.join(ROOT, "tests", "golden", fname))  # allow_pickle=False (default)
        for b in meta["batches"]:
            nm = b["name"]
            pairs = np.ascontiguousarray(z[f"{nm}_pairs"]).view(bswgen.SEQPAIR_DTYPE).reshape(-1).copy()
            out.append((nm, pairs, z[f"{nm}_ref"], z[f"{nm}_qer"], b["w"], b["scoring"]))
    return out


@pytest.fixture(scope="session")
def golden():
    return load_golden()
