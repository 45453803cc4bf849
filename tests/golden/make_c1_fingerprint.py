"""Container-side: pin bwa-mem2-arm_amd/py/c1data.py to the reference's own C1 generator.

Runs the two Python heredocs of /root/reference/benchmark_threading.sh (lines 42-70; read from
the reference at run time, never stored here) in a scratch directory, checks that c1data's
regenerated reference and reads equal the FASTA / FASTQ they write, and records digests of
both in tests/golden/c1_fingerprint.json (which the CPU tests check c1data against)."""

import hashlib
import json
import os
import re
import subprocess
import sys
import tempfile

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, os.path.join(ROOT, "bwa-mem2-arm_amd", "py"))
import c1data  # noqa: E402


def main():
    sh = open("/root/reference/benchmark_threading.sh").read()
    blocks = re.findall(r"python3 << 'EOF'\n(.*?)\nEOF", sh, re.S)
    assert len(blocks) == 2
    with tempfile.TemporaryDirectory() as d:
        os.makedirs(os.path.join(d, "test_data"))
        for b in blocks:
            subprocess.run([sys.executable, "-c", b], check=True, cwd=d)
        fa = open(os.path.join(d, "test_data", "test_ref.fa"), "rb").read()
        fq = open(os.path.join(d, "test_data", "test_reads.fq"), "rb").read()
    ref, reads, off, lens, starts = c1data.workload()
    seq = b"".join(fa.split(b"\n")[1:]).decode()
    assert seq == "".join("ACGT"[c] for c in ref), "reference differs from the reference's generator"
    rl = fq.split(b"\n")
    for i in range(c1data.N_READS):
        assert rl[4 * i + 1].decode() == "".join("ACGT"[c] for c in reads[i * 150:(i + 1) * 150]), i
    fp = c1data.fingerprint(ref, starts)
    fp.update(source="/root/reference/benchmark_threading.sh:42-70 (run here, outputs compared)",
              reference_fasta_sha256=hashlib.sha256(fa).hexdigest(),
              reference_fastq_sha256=hashlib.sha256(fq).hexdigest())
    json.dump(fp, open(os.path.join(HERE, "c1_fingerprint.json"), "w"), indent=1)
    print(fp)


if __name__ == "__main__":
    main()
