import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (gfx950) GPU; parity tests through the C ABI")


@pytest.fixture(scope="session", autouse=True)
def _built():
    """Make sure the in-tree libraries exist (build() is idempotent and fast when up to date)."""
    import __graft_entry__ as g

    g.build()
    yield


GOLDEN = os.path.join(ROOT, "tests", "golden")


def irregular_families(seed, n_parents, L, fam=6, p_sub=0.08, p_n=0.05, p_lower=0.03, p_len=0.05, alphabet=b"ACGT",
                       p_utf8=0.0):
    """UMI families whose members carry substitutions, N, lowercase bytes and length
    changes at high rates, so Hamming-1 edges join irregular strings to regular codes,
    to each other, and bridge regular clusters (the H3.2 spec).
    p_utf8 > 0: members also get two bytes replaced by the 2-byte UTF-8 char U+00E9
    (same byte length, one char fewer) or, half as often, one byte replaced by it (one
    byte longer), and the pin pair A^(L-2)+U+00E9 / A^L is appended: H2.1 distance 1
    (chars zipped), 2 byte mismatches, so H3 (byte-wise) draws no edge between them."""
    import numpy as np

    rng = np.random.default_rng(seed)
    out = []
    for _ in range(n_parents):
        parent = bytearray(rng.choice(list(alphabet), size=L).astype(np.uint8).tobytes())
        for _ in range(int(rng.integers(1, fam + 1))):
            u = bytearray(parent)
            for q in range(L):
                r = rng.random()
                if r < p_sub:
                    u[q] = int(rng.choice(list(alphabet)))
                elif r < p_sub + p_n:
                    u[q] = ord("N")
                elif r < p_sub + p_n + p_lower:
                    u[q] = u[q] | 0x20
            if p_utf8 > 0 and len(u) >= 2:
                r = rng.random()
                if r < p_utf8:
                    q = int(rng.integers(0, len(u) - 1))
                    u[q:q + 2] = b"\xc3\xa9"
                elif r < 1.5 * p_utf8:
                    q = int(rng.integers(0, len(u)))
                    u[q:q + 1] = b"\xc3\xa9"
            r = rng.random()
            if r < p_len / 2:
                u = u[:-1]
            elif r < p_len:
                u = u + b"A"
            out.append(bytes(u))
    out += [None, b"", b"N" * L, b"n" * L]
    if p_utf8 > 0 and L >= 2:
        out += [b"A" * (L - 2) + "\u00e9".encode(), b"A" * L]
    return out
