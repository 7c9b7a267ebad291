"""CPU check of the repeat certificate's argument (kmer_kernels.hip
may_repeat16): a row where no aligned 16-mer [16j, 16j + 16) occurs again at a later
position holds no k-mer twice for k >= 31. Brute force over random rows with planted
tandem repeats and copied segments (the GPU bit itself is pinned against the same
restatement in tests/test_gpu_c3.py::test_repeat_certificate_bit)."""
import random


def norep(row: str) -> bool:
    L = len(row)
    for a in range(0, L - 15, 16):
        s = row[a:a + 16]
        for i in range(a + 1, L - 15):
            if row[i:i + 16] == s:
                return False
    return True


def has_repeat(row: str, k: int) -> bool:
    seen = set()
    for p in range(len(row) - k + 1):
        x = row[p:p + k]
        if x in seen:
            return True
        seen.add(x)
    return False


def test_certificate_is_sound_for_k31_k32():
    rnd = random.Random(1)
    certified = 0
    for _ in range(2500):
        L = rnd.randint(31, 224)
        r = [rnd.choice("ACGT") for _ in range(L)]
        x = rnd.random()
        if x < 0.4:  # tandem repeat of a 1-70 base unit
            u = rnd.randint(1, 70)
            r = (r[:u] * (L // u + 1))[:L]
        elif x < 0.8:  # a copied segment of 16-60 bases
            a, b, n = rnd.randint(0, L - 1), rnd.randint(0, L - 1), rnd.randint(16, 60)
            for t in range(n):
                if a + t < L and b + t < L:
                    r[b + t] = r[a + t]
        row = "".join(r)
        c = norep(row)
        certified += c
        for k in (31, 32):
            assert not (c and has_repeat(row, k)), (row, k)
    assert certified > 400


def test_certificate_not_sound_below_k31():
    """k = 30 is outside the argument (k - 15 < 16): a row can hold a 30-mer twice with no
    aligned 16-mer repeated, which is why the spectrum call requires k_eff 32."""
    rnd = random.Random(7)
    found = False
    for _ in range(20000):
        base = "".join(rnd.choice("ACGT") for _ in range(120))
        d = rnd.randint(31, 60)
        p = rnd.randint(0, 30)
        row = list(base)
        for t in range(30):
            row[p + d + t] = row[p + t]
        row = "".join(row)
        if norep(row) and has_repeat(row, 30):
            found = True
            break
    assert found
