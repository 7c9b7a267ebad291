"""H4.4 + H5 graph assembly: the product (GPU spectra + host C++ graph code in
librogtk_hip.so) vs the pure-Python restatement (oracle/pyassembly.py), exact strings.

Pinned against the reference itself: the expected contig in the comment of its
test at fracture.rs:611 (shortest_path, k=13) and the empty result for absent
anchors (fracture.rs:684-707). Node-order-dependent choices (ties between equally
long contigs, Dijkstra ties) follow ascending k-mer order in both implementations;
the reference's MPHF order is not reproducible (parity unpinned there).
"""
from __future__ import annotations

import numpy as np
import pyarrow as pa
import pytest

pytestmark = pytest.mark.gpu

REF_SEQS = [b"GAGACTGCATGGGCTGGTGGGCGTCCGTCTGC", b"GGGCTGGTGGGCGTCCGTCTGCTTTAGTGAGGGT"]
FASTA = [  # fracture.rs:573-586 create_test_fasta
    b"ATGCATGCATGCTAGCTGATCGATCGTAGCTAGCTAGCTGATCGATCGTACGTACGTACGTAGCTACGTACGTACGTAGCTAGCTGATCGTAGCTACGTAGCTAGCTAGCTGATCGTACGTACGT",
    b"GTAGCTAGCTAGCTGATCGATCGTACGTACGTACGTAGCTACGTACGTACGTAGCTAGCTGATCGTAGCTACGTAGCTAGCTAGCTGATCGTACGTACGTAGCTGATCGATCGTAGCTACGTACGT",
    b"GTACGTACGTACGTAGCTACGTACGTACGTAGCTAGCTGATCGTAGCTACGTAGCTAGCTAGCTGATCGTACGTACGTAGCTGATCGATCGTAGCTACGTACGTACGTAGCTACGTACGTACGTAG",
    b"TACGTACGTACGTAGCTAGCTGATCGTAGCTACGTAGCTAGCTAGCTGATCGTACGTACGTAGCTGATCGATCGTAGCTACGTACGTACGTAGCTACGTACGTACGTAGCTAGCTGATCGTAGCT",
]


@pytest.fixture(scope="module")
def rg():
    import rogtk_amd
    return rogtk_amd


def A():
    from oracle import pyassembly
    return pyassembly


def _col(items):
    return pa.array(items, type=pa.large_binary())


def _same(rg, items, k, mc, method, sa=None, ea=None, min_length=None, auto_k=False):
    got = rg.assemble_sequences(_col(items), k, mc, method, sa, ea, min_length, auto_k=auto_k)
    ref = A().assemble(items, k, mc, method, sa, ea, True, min_length, auto_k)
    assert got == "\n".join(ref), (k, mc, method)
    return got


def test_reference_shortest_path_kat(rg):
    """fracture.rs:611 / :630-681: the two test reads assemble to the 44-bp contig."""
    got = _same(rg, REF_SEQS, 13, 1, "shortest_path", "GAGACTGCATGG", "TTTAGTGAGGGT")
    assert got == "GAGACTGCATGGGCTGGTGGGCGTCCGTCTGCTTTAGTGAGGGT"


def test_reference_invalid_anchors(rg):
    """fracture.rs:684-707: anchors absent from the graph -> no contig."""
    got = _same(rg, [b"AAAACCCCCAAAAA", b"TTTTTGGGGGTTTT"], 4, 1, "shortest_path", "NONEXISTENT", "ALSONOTHERE")
    assert got == ""


def test_reference_compare_methods(rg):
    """fracture.rs:710-761 at k=4: compression yields a contig. (Its shortest_path half
    asserts a contig although 12-bp anchors cannot prefix a 4-mer node of the
    uncompressed graph the reference searches; the restated code yields none.)"""
    assert _same(rg, REF_SEQS, 4, 1, "compression") != ""
    assert _same(rg, REF_SEQS, 4, 1, "shortest_path", "GAGACTGCATGG", "TTTAGTGAGGGT") == ""


def test_reference_fasta_reads(rg):
    """fracture.rs:595-607 reads at k=20 (effective 32): a tail entering a cycle gives
    two unitigs (the test's >150-bp expectation needs effective k 64: k=33 -> 189 bp)."""
    assert len(_same(rg, FASTA, 20, 1, "compression")) == 125
    assert len(_same(rg, FASTA, 33, 1, "compression")) == 189
    _same(rg, FASTA, 20, 1, "shortest_path_auto")


def _family(rng, n_reads, tpl_len, read_len, p_err):
    tpl = bytes(rng.choice(np.frombuffer(b"ACGT", np.uint8), tpl_len))
    out = []
    for _ in range(n_reads):
        a = int(rng.integers(0, max(1, tpl_len - read_len)))
        r = bytearray(tpl[a:a + read_len])
        for j in range(len(r)):
            if rng.random() < p_err:
                r[j] = b"ACGT"[int(rng.integers(4))]
        out.append(bytes(r))
    return tpl, out


@pytest.mark.parametrize("seed", range(6))
@pytest.mark.parametrize("method", ["compression", "shortest_path", "shortest_path_auto"])
def test_random_families(rg, seed, method):
    rng = np.random.default_rng(seed)
    tpl, reads = _family(rng, int(rng.integers(8, 30)), int(rng.integers(80, 220)), int(rng.integers(40, 90)), 0.01)
    reads += [None, b"ACGTN" * 5, b"acgt" * 6]
    sa, ea = (tpl[:10].decode(), tpl[-10:].decode()) if method == "shortest_path" else (None, None)
    for k, mc in ((5, 1), (9, 2), (13, 1), (17, 3), (21, 2), (33, 1)):
        _same(rg, reads, k, mc, method, sa, ea)
    _same(rg, reads, 0, 2, method, sa, ea, auto_k=True)
    _same(rg, reads, 13, 1, method, sa, ea, min_length=60)


def test_sweep_and_optimize(rg):
    rng = np.random.default_rng(42)
    tpl, reads = _family(rng, 25, 150, 70, 0.005)
    sa, ea = tpl[:10].decode(), tpl[-10:].decode()
    got = rg.sweep_assembly_params(_col(reads), 5, 21, 4, 1, 7, 3, "shortest_path", sa, ea)
    ref = A().sweep(reads, 5, 21, 4, 1, 7, 3, "shortest_path", sa, ea)
    assert list(zip(*(got.field(f).to_pylist() for f in ("k", "min_coverage", "contig_length")))) == ref
    for explore, prio in ((False, False), (True, False), (True, True)):
        g = rg.optimize_assembly(_col(reads), "shortest_path", sa, ea, start_k=11, start_min_coverage=4,
                                 max_iterations=6, explore_k=explore, prioritize_length=prio)
        r = A().optimize(reads, "shortest_path", sa, ea, 11, 4, 6, explore, prio)
        assert g == r, (explore, prio)


def test_method_errors(rg):
    from rogtk_amd import RogtkError

    with pytest.raises(RogtkError, match="should not be provided for compression"):
        rg.assemble_sequences(_col(REF_SEQS), 13, 1, "compression", "AC", "GT")
    with pytest.raises(RogtkError, match="Both start_anchor and end_anchor are required"):
        rg.assemble_sequences(_col(REF_SEQS), 13, 1, "shortest_path", "AC", None)
    with pytest.raises(RogtkError, match="Invalid assembly method"):
        rg.assemble_sequences(_col(REF_SEQS), 13, 1, "bogus")
    got = rg.assemble_sequences_with_anchors(_col(REF_SEQS), ["GAGACTGCATGG"], ["TTTAGTGAGGGT"], k=13, min_coverage=1)
    assert got == "GAGACTGCATGGGCTGGTGGGCGTCCGTCTGCTTTAGTGAGGGT"


def _c3_groups(n, seed_rows=None):
    """n synth-v1 150-bp reads with 12-bp UMIs on the device, their exact H3 ids (the
    caller's group_by('umi'), rogtk/__init__.py:206-214)."""
    import torch

    from rogtk_amd import device as D
    from rogtk_amd import synth

    codes = torch.from_numpy(synth.umi_codes(n, 12).view(np.int32)).cuda()
    reads_h = synth.reads(n, 150)
    values = torch.from_numpy(reads_h.reshape(-1)).cuda()
    offsets = torch.arange(0, (n + 1) * 150, 150, dtype=torch.int64, device="cuda")
    eng = D.ClusterEngine(12, min(n, 4 ** 12), "cuda")
    cid = torch.empty(n, dtype=torch.int32, device="cuda")
    D.cluster_batch(eng, D.PackedBatch(codes, 12), cid, 0)
    return reads_h, values, offsets, cid


@pytest.mark.parametrize("k,mc,method,n,sample", [(15, 5, "compression", 1_000_000, 2000),
                                                  (10, 5, "shortest_path_auto", 200_000, 400),
                                                  (17, 3, "compression", 200_000, 400)])
def test_batched_groups_match_per_group(rg, k, mc, method, n, sample):
    """Round 6, batched H5 (rogtk_assemble_groups_host over a whole group_spectra result):
    every group's string identical to the per-group rogtk_assemble_host call (its own GPU
    spectrum at min_coverage 0, CountFilter + censoring on the host) on a sample of the C3
    groups (the largest ones included), and to the Python restatement on a smaller one."""
    import torch

    from rogtk_amd import assembly as AS

    reads_h, values, offsets, cid = _c3_groups(n)
    rows, go, arr, nc = AS.assemble_column_groups(offsets, values, cid, k, mc, method)
    torch.cuda.synchronize()
    G = len(go) - 1
    assert len(arr) == G and len(nc) == G
    rows_h, goh = rows.cpu().numpy(), go.cpu().numpy()
    sizes = np.diff(goh)
    rng = np.random.default_rng(k + mc)
    pick = np.unique(np.concatenate([rng.choice(G, size=sample, replace=False), np.argsort(sizes)[-50:]]))
    got = arr.to_pylist()
    nonempty = 0
    for j, g in enumerate(pick):
        items = [bytes(reads_h[r]) for r in rows_h[goh[g]:goh[g + 1]]]
        want = rg.assemble_sequences(_col(items), k, mc, method)
        assert got[g] == want, (g, len(items))
        assert nc[g] == (want.count("\n") + 1 if want else 0)
        nonempty += bool(want)
        if j < 60:  # the Python restatement (only_largest, as the expression)
            assert got[g] == "\n".join(A().assemble(items, k, mc, method, None, None, True, None, False)), g
    assert nonempty > len(pick) // 2
