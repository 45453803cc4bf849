"""BASELINE configs[0] (C1): the reference's own synthetic data, regenerated bit-exactly.

The reference's threading benchmark builds its test data with CPython's `random` module
(/root/reference/benchmark_threading.sh:42-70): a 1,000,000-base reference drawn with
`choices` over A, C, G, T after `seed(42)`, written as FASTA and read back, then -- in a fresh
interpreter, seeded with 42 again -- 10,000 exact 150-base single-end reads, read i starting at
`randint(0, len(ref) - 150)`.  This module makes the same calls in the same order on the same
generator (CPython's Mersenne Twister, which the GPU box's interpreter shares), so the
sequences are the reference's own; `tests/golden/c1_fingerprint.json` pins their digests.
Codes follow bwa's nt4 table (A 0, C 1, G 2, T 3)."""

from __future__ import annotations

import hashlib
import random

import numpy as np

REF_LEN = 1_000_000
N_READS = 10_000
READ_LEN = 150
_CODE = {"A": 0, "C": 1, "G": 2, "T": 3}


def reference() -> np.ndarray:
    """The 1 Mb reference as codes 0..3 (the first heredoc of benchmark_threading.sh)."""
    rng = random.Random()
    rng.seed(42)
    seq = "".join(rng.choices(["A", "C", "G", "T"], k=REF_LEN))
    return np.frombuffer(seq.translate(str.maketrans("ACGT", "\x00\x01\x02\x03")).encode("latin-1"),
                         dtype=np.uint8).copy()


def read_starts(ref_len: int = REF_LEN) -> np.ndarray:
    """Read start positions (the second heredoc: a fresh seed(42), one randint per read)."""
    rng = random.Random()
    rng.seed(42)
    return np.array([rng.randint(0, ref_len - READ_LEN) for _ in range(N_READS)], dtype=np.int64)


def workload():
    """(ref codes, reads concatenated, read_off, read_len, starts): 10K exact 150-bp SE reads."""
    ref = reference()
    starts = read_starts(len(ref))
    idx = starts[:, None] + np.arange(READ_LEN)[None, :]
    reads = ref[idx].reshape(-1).copy()
    off = np.arange(N_READS, dtype=np.int64) * READ_LEN
    lens = np.full(N_READS, READ_LEN, dtype=np.int32)
    return ref, reads, off, lens, starts


def fingerprint(ref: np.ndarray, starts: np.ndarray) -> dict:
    return {"ref_sha256": hashlib.sha256(ref.tobytes()).hexdigest(),
            "starts_sha256": hashlib.sha256(starts.astype("<i8").tobytes()).hexdigest(),
            "ref_head": "".join("ACGT"[c] for c in ref[:60]), "first_starts": [int(x) for x in starts[:8]]}
