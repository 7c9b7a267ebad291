"""The polars plugin ABI of librogtk_hip.so (rogtk_amd/csrc/polars_plugin.cpp), driven the
way polars drives it (Arrow C Data Interface + polars-ffi SeriesExport + pickled kwargs).

CPU tests: exported symbols, version, output fields, kwargs pickle reader, argument and
dtype errors (all raised before any device work). GPU tests: every expression against the
eager pyarrow API (itself parity-tested against the oracle) and the oracle directly, over
polars' own Utf8View layout and the Utf8 / LargeUtf8 layouts, multi-chunk and sliced
inputs with nulls.
"""
import math
import pickle
import subprocess

import numpy as np
import pyarrow as pa
import pytest

from rogtk_amd import _lib, plugin

SYMBOLS = ["_polars_plugin_get_version", "_polars_plugin_get_last_error_message"]
for _n in plugin.EXPRESSIONS:
    SYMBOLS += ["_polars_plugin_" + _n, "_polars_plugin_field_" + _n]

F64 = ("shannon_entropy", "linguistic_complexity", "homopolymer_fraction", "dinucleotide_entropy", "dust_score",
       "combined_score")
SINGLE = {
    "umi_shannon_entropy_expr": "shannon_entropy",
    "umi_linguistic_complexity_expr": "linguistic_complexity",
    "umi_homopolymer_fraction_expr": "homopolymer_fraction",
    "umi_dinucleotide_entropy_expr": "dinucleotide_entropy",
    "umi_combined_score_expr": "combined_score",
    "umi_longest_homopolymer_expr": "longest_homopolymer_run",
    "umi_dust_score_expr": "dust_score",
}


# ------------------------------------------------------------------ CPU
def test_library_exports_every_plugin_symbol():
    out = subprocess.run(["nm", "-D", "--defined-only", _lib.HIP_LIB_PATH], capture_output=True, text=True,
                         check=True).stdout
    have = {ln.split()[-1] for ln in out.splitlines() if ln.strip()}
    missing = [s for s in SYMBOLS if s not in have]
    assert not missing, missing


def test_package_dir_holds_exactly_one_shared_library():
    # polars resolves plugin_path=<package dir> to the first shared library found there
    import os
    libs = [f for f in os.listdir(plugin.PLUGIN_PATH) if f.endswith((".so", ".dll", ".pyd"))]
    assert libs == ["librogtk_hip.so"], libs


def test_plugin_version():
    assert plugin.plugin_version() == 1  # polars-ffi (major 0, minor 1)


@pytest.mark.parametrize("name,typ", [
    ("umi_complexity_all_expr", pa.struct([("shannon_entropy", pa.float64()), ("linguistic_complexity", pa.float64()),
                                           ("homopolymer_fraction", pa.float64()),
                                           ("dinucleotide_entropy", pa.float64()),
                                           ("longest_homopolymer_run", pa.uint32()), ("dust_score", pa.float64()),
                                           ("combined_score", pa.float64())])),
    ("umi_shannon_entropy_expr", pa.float64()),
    ("umi_longest_homopolymer_expr", pa.uint32()),
    ("hamming_distance_expr", pa.uint32()),
    ("hamming_within_expr", pa.bool_()),
    ("assemble_sequences_expr", pa.string_view()),
    ("assemble_sequences_with_anchors_expr", pa.string_view()),
    ("sweep_assembly_params_expr", pa.struct([("k", pa.int64()), ("min_coverage", pa.int64()),
                                              ("contig_length", pa.int64())])),
    ("optimize_assembly_expr", pa.struct([("contig", pa.string_view()), ("k", pa.uint32()),
                                          ("min_coverage", pa.uint32()), ("length", pa.uint32()),
                                          ("input_sequences", pa.uint32())])),
    ("reverse_complement_series", pa.string_view()),
    ("parse_cigar_series", pa.string_view()),
    ("cigar_aligned_ref_expr", pa.string_view()),
    ("cigar_aligned_query_expr", pa.string_view()),
    ("extract_cigar_insertions_expr", pa.string_view()),
    ("enrich_allele_insertions_expr", pa.string_view()),
    ("phred_to_numeric_series_str", pa.string_view()),
    ("phred_to_numeric_series", pa.large_list(pa.uint8())),
])
def test_output_fields(name, typ):
    f = plugin.call_plugin_field(name, [pa.field("umi", pa.string_view())])
    assert f.name == "umi" and f.type == typ


def test_kwargs_pickle_reader():
    kw = {"target": "ACGT", "max_distance": 3, "neg": -5, "big": 2 ** 40, "none": None, "t": True, "f": False,
          "x": 0.25, "lst": [1, "a"], "tup": (1, 2), "u": "μ-unicode", "k" * 300: "long key",
          "s": "x" * 70000}
    for proto in (2, 3, 4, 5):
        got = plugin.kwargs_as_parsed(raw=pickle.dumps(kw, protocol=proto))
        lines = dict(ln.split("=", 1) for ln in got.splitlines())
        assert lines["target"] == "'ACGT'" and lines["max_distance"] == "3" and lines["neg"] == "-5"
        assert lines["big"] == str(2 ** 40) and lines["none"] == "None"
        assert lines["t"] == "True" and lines["f"] == "False" and float(lines["x"]) == 0.25
        assert lines["lst"] == "[1, 'a']" and lines["tup"] == "[1, 2]"
        assert lines["u"] == "'μ-unicode'" and lines["k" * 300] == "'long key'" and len(lines["s"]) == 70002
    # memoised (shared) string objects come back through BINGET
    shared = "ACGTAC"
    got = plugin.kwargs_as_parsed(raw=pickle.dumps({"a": shared, "b": shared}, protocol=2))
    assert got == "a='ACGTAC'\nb='ACGTAC'\n"
    assert plugin.kwargs_as_parsed(raw=b"") == ""
    with pytest.raises(_lib.RogtkError, match="truncated"):
        plugin.kwargs_as_parsed(raw=pickle.dumps({"a": "xyz"}, protocol=5)[:-4])


def _err(name, inputs, kwargs=None):
    with pytest.raises(_lib.RogtkError) as ei:
        plugin.call_plugin(name, inputs, kwargs)
    return str(ei.value)


def test_errors_cross_the_plugin_abi_and_inputs_are_released():
    umis = pa.array(["ACGT"], type=pa.string_view())
    # serde: HammingKwargs.target is required (expressions.rs:1016-1020)
    assert "missing field `target`" in _err("hamming_distance_expr", [umis], {"max_distance": 1})
    assert "missing field `target`" in _err("hamming_within_expr", [umis], None)
    # inputs[0].str()? on a non-string series
    assert "expected `String`, got `i64`" in _err("umi_complexity_all_expr", [pa.array([1, 2])])
    assert "expected `String`, got `binary`" in _err("umi_shannon_entropy_expr", [pa.array([b"A"])])
    # assemble_sequences_expr method / anchor validation (expressions.rs:700-730)
    base = {"k": 13, "min_coverage": 1}
    assert "Anchor sequences should not be provided for compression method" in _err(
        "assemble_sequences_expr", [umis], dict(base, method="compression", start_anchor="ACG"))
    assert "Both start_anchor and end_anchor are required for shortest_path method" in _err(
        "assemble_sequences_expr", [umis], dict(base, method="shortest_path", start_anchor="ACG", end_anchor=None))
    assert "Invalid assembly method" in _err("assemble_sequences_expr", [umis], dict(base, method="bogus"))
    assert "missing field `k`" in _err("assemble_sequences_expr", [umis], {"method": "compression",
                                                                            "min_coverage": 1})
    # with_anchors (expressions.rs:776-825)
    anc = pa.array(["ACG"], type=pa.string_view())
    assert "requires 3 inputs" in _err("assemble_sequences_with_anchors_expr", [umis, anc],
                                       dict(base, method="shortest_path"))
    assert "start_anchor column is empty" in _err(
        "assemble_sequences_with_anchors_expr", [umis, pa.array([None], type=pa.string_view()), anc],
        dict(base, method="shortest_path"))
    assert "not supported with dynamic anchors" in _err("assemble_sequences_with_anchors_expr", [umis, anc, anc],
                                                        dict(base, method="compression"))
    # optimize_assembly_expr (fracture_opt.rs:298-304)
    assert "start_anchor is required" in _err("optimize_assembly_expr", [umis],
                                              {"method": "shortest_path", "start_k": 31, "start_min_coverage": 1})


# ------------------------------------------------------------------ GPU
def _layouts(values, chunks=3):
    """The same column as Utf8View (polars' String), Utf8, LargeUtf8, multi-chunk and sliced."""
    out = {}
    for tname, t in (("view", pa.string_view()), ("utf8", pa.string()), ("large", pa.large_string())):
        out[tname] = pa.array(values, type=t)
    n = len(values)
    cut = [0] + sorted({n * (i + 1) // chunks for i in range(chunks - 1)}) + [n]
    out["chunked_view"] = pa.chunked_array([pa.array(values[a:b], type=pa.string_view()) for a, b in zip(cut, cut[1:])],
                                           type=pa.string_view())
    big = pa.array(["GG"] * 3 + list(values) + ["TT"] * 5, type=pa.string_view())
    out["sliced_view"] = big.slice(3, n)
    big2 = pa.array(["GG"] * 5 + list(values) + ["TT"], type=pa.string())
    out["sliced_utf8"] = big2.slice(5, n)
    return out


def _umis():
    from rogtk_amd import synth
    vals = [bytes(u).decode("latin-1") for u in synth.umi_ascii(3000, 12, p_n=5e-3, p_lower=2e-3)]
    vals[3] = None
    vals[10] = ""
    vals[11] = "ACGTACGTACGTACGTAACC"  # > 12 bytes: out-of-line view
    vals[12] = "ACGT" * 20
    vals[13] = "ACGTμACGTAC"
    for i in range(100, 3000, 97):
        vals[i] = None
    return vals


def _bits(a):
    a = np.asarray(a)
    return a.view(np.uint64) if a.dtype == np.float64 else a


@pytest.mark.gpu
def test_umi_complexity_all_expr_matches_api():
    import rogtk_amd as rg
    vals = _umis()
    ref = rg.umi_complexity_scores(pa.array(vals, type=pa.large_string()))
    ref = ref.combine_chunks() if isinstance(ref, pa.ChunkedArray) else ref
    valid = np.array([v is not None for v in vals])
    for lname, col in _layouts(vals).items():
        got, name = plugin.call_plugin_named("umi_complexity_all_expr", [col], names=["umi"])
        assert name == "umi"
        got = got.combine_chunks()
        assert got.null_count == 0, "struct rows stay valid (df.into_struct); the fields carry the nulls"
        for f, _ in rg.FIELDS:
            g, r = got.field(f), ref.field(f)
            assert np.array_equal(np.asarray(g.is_valid()), valid), (lname, f)
            gv = _bits(g.fill_null(0).to_numpy(zero_copy_only=False))
            rv = _bits(r.fill_null(0).to_numpy(zero_copy_only=False))
            assert np.array_equal(gv[valid], rv[valid]), (lname, f)


@pytest.mark.gpu
@pytest.mark.parametrize("expr", sorted(SINGLE))
def test_single_field_exprs_match_api(expr):
    import rogtk_amd as rg
    vals = _umis()
    field = SINGLE[expr]
    ref = rg.umi_complexity(pa.array(vals, type=pa.large_string()), (field,))[field]
    ref = ref.combine_chunks() if isinstance(ref, pa.ChunkedArray) else ref
    for lname, col in _layouts(vals).items():
        got, name = plugin.call_plugin_named(expr, [col], names=["u"])
        assert name == "u"
        got = got.combine_chunks()
        assert got.type == ref.type and got.null_count == ref.null_count, lname
        assert np.array_equal(_bits(got.fill_null(0).to_numpy(zero_copy_only=False)),
                              _bits(ref.fill_null(0).to_numpy(zero_copy_only=False))), lname


@pytest.mark.gpu
def test_umi_exprs_match_oracle_and_reference_kats():
    from oracle import pyoracle as P
    kat = ["AAAAAAAAAAAA", "ACGTACGTACGT", "AACCGGTTAACC", "ACGTTGCAACGT", "GATTACAGATTA", "NNNNNNNNNNNN",
           "ACGTNACGTACG", "acgtacgtacgt", ""]
    got = plugin.call_plugin("umi_complexity_all_expr", [pa.array(kat, type=pa.string_view())]).combine_chunks()
    ref = P.umi_complexity(P.StrCol.from_list([s.encode() for s in kat]))
    for f in F64:
        g = got.field(f).to_numpy(zero_copy_only=False)
        r = ref[f]
        assert np.array_equal(g[:-1].view(np.uint64), r[:-1].view(np.uint64)), f
    assert math.isnan(got.field("combined_score")[8].as_py())  # len 0: 0/0 (umi_score.rs:31)
    assert got.field("combined_score")[0].as_py() == 0.125


@pytest.mark.gpu
@pytest.mark.parametrize("target", ["ACGTACGTACGT", "AAAAAAAAAAAA", "ACGT", "", "ACGTμACGTAC"])
@pytest.mark.parametrize("maxd", [None, 0, 2])
def test_hamming_exprs_match_api(target, maxd):
    import rogtk_amd as rg
    vals = _umis()
    rd = rg.hamming_distance(pa.array(vals, type=pa.large_string()), target)
    rw = rg.hamming_within(pa.array(vals, type=pa.large_string()), target, 1 if maxd is None else maxd)
    rd = rd.combine_chunks() if isinstance(rd, pa.ChunkedArray) else rd
    rw = rw.combine_chunks() if isinstance(rw, pa.ChunkedArray) else rw
    for lname, col in _layouts(vals).items():
        gd = plugin.call_plugin("hamming_distance_expr", [col], {"target": target}).combine_chunks()
        kw = {"target": target, "max_distance": maxd}
        gw = plugin.call_plugin("hamming_within_expr", [col], kw).combine_chunks()
        assert gd.equals(rd), lname
        assert gw.equals(rw), lname


def _family(seed, n_reads=40, tpl_len=160, read_len=90):
    rng = np.random.default_rng(seed)
    tpl = "".join(rng.choice(list("ACGT"), tpl_len))
    reads = []
    for _ in range(n_reads):
        a = int(rng.integers(0, tpl_len - read_len + 1))
        reads.append(tpl[a:a + read_len])
    return tpl, reads


@pytest.mark.gpu
@pytest.mark.parametrize("method", ["compression", "shortest_path", "shortest_path_auto"])
def test_assemble_sequences_expr_matches_api(method):
    import rogtk_amd as rg
    for seed in range(4):
        tpl, reads = _family(seed)
        reads_n = reads[:5] + [None] + reads[5:]
        anchors = {"start_anchor": tpl[:8], "end_anchor": tpl[-8:]} if method == "shortest_path" else {}
        for k, cov in ((13, 1), (17, 2), (31, 3)):
            ref = rg.assemble_sequences(pa.array(reads, type=pa.large_string()), k=k, min_coverage=cov,
                                        method=method, **anchors)
            kw = {"k": k, "min_coverage": cov, "method": method, "start_anchor": None, "end_anchor": None,
                  "min_length": None, "export_graphs": False, "only_largest": False, "auto_k": False,
                  "prefix": None}
            kw.update(anchors)
            col = pa.chunked_array([pa.array(reads_n[:7], type=pa.string_view()),
                                    pa.array(reads_n[7:], type=pa.string_view())])
            got, name = plugin.call_plugin_named("assemble_sequences_expr", [col], kw, names=["seq"])
            assert name == "assembled_sequences"
            assert got.type == pa.string_view() and len(got) == 1
            assert got[0].as_py() == ref, (seed, k, cov)


@pytest.mark.gpu
def test_assemble_with_anchors_and_reference_kat():
    import rogtk_amd as rg
    # the reference's own expected contig (src/fracture.rs:611, test reads :630-681)
    seqs = ["GAGACTGCATGGGCTGGTGGGCGTCCGTCTGC", "GGGCTGGTGGGCGTCCGTCTGCTTTAGTGAGGGT"]
    kw = {"k": 13, "min_coverage": 1, "method": "shortest_path", "start_anchor": None, "end_anchor": None,
          "min_length": None, "export_graphs": False, "only_largest": False, "auto_k": False, "prefix": None}
    got = plugin.call_plugin("assemble_sequences_with_anchors_expr",
                             [pa.array(seqs, type=pa.string_view()), pa.array(["GAGACTGCATGG"], type=pa.string_view()),
                              pa.array(["TTTAGTGAGGGT"], type=pa.string_view())], kw)
    assert got[0].as_py() == "GAGACTGCATGGGCTGGTGGGCGTCCGTCTGCTTTAGTGAGGGT"
    tpl, reads = _family(11)
    s_col = pa.array([tpl[:10], "IGNORED"], type=pa.string_view())
    e_col = pa.array([tpl[-10:], None], type=pa.string_view())
    kw = {"k": 17, "min_coverage": 1, "method": "shortest_path", "start_anchor": None, "end_anchor": None,
          "min_length": None, "export_graphs": False, "only_largest": False, "auto_k": False, "prefix": None}
    got = plugin.call_plugin("assemble_sequences_with_anchors_expr",
                             [pa.array(reads, type=pa.string_view()), s_col, e_col], kw)
    ref = rg.assemble_sequences_with_anchors(pa.array(reads, type=pa.large_string()), [tpl[:10]], [tpl[-10:]],
                                             k=17, min_coverage=1)
    assert got[0].as_py() == ref


@pytest.mark.gpu
def test_sweep_and_optimize_exprs_match_api():
    import rogtk_amd as rg
    tpl, reads = _family(5, n_reads=60)
    col = pa.array(reads, type=pa.string_view())
    kw = {"k_start": 9, "k_end": 33, "k_step": 4, "cov_start": 1, "cov_end": 4, "cov_step": 1,
          "method": "compression", "start_anchor": None, "end_anchor": None, "min_length": None,
          "export_graphs": False, "prefix": None, "auto_k": False}
    got, name = plugin.call_plugin_named("sweep_assembly_params_expr", [col], kw, names=["seq"])
    ref = rg.sweep_assembly_params(pa.array(reads, type=pa.large_string()), k_start=9, k_end=33, k_step=4,
                                   cov_start=1, cov_end=4, cov_step=1, method="compression")
    assert name == "seq"
    assert got.combine_chunks().equals(ref)
    okw = {"method": "shortest_path", "start_anchor": tpl[:9], "end_anchor": tpl[-9:], "start_k": 31,
           "start_min_coverage": 1, "min_length": None, "export_graphs": False, "prefix": None,
           "max_iterations": None, "explore_k": None, "prioritize_length": None}
    got = plugin.call_plugin("optimize_assembly_expr", [col], okw).combine_chunks()
    ref = rg.optimize_assembly(pa.array(reads, type=pa.large_string()), start_anchor=tpl[:9], end_anchor=tpl[-9:])
    row = got[0].as_py()
    assert row == ref


@pytest.mark.gpu
def test_empty_and_all_null_columns():
    for t in (pa.string_view(), pa.string(), pa.large_string()):
        got = plugin.call_plugin("umi_complexity_all_expr", [pa.array([], type=t)])
        assert len(got) == 0
        got = plugin.call_plugin("hamming_distance_expr", [pa.array([None, None], type=t)], {"target": "AC"})
        assert got.to_pylist() == [None, None]


@pytest.mark.gpu
def test_string_exprs_match_oracle():
    """The element-wise string expressions through the plugin ABI (Utf8View / Utf8 /
    LargeUtf8, chunked, sliced) equal the oracle restatement."""
    from oracle import pystrings as O

    rng = np.random.default_rng(9)
    n = 600
    al = np.frombuffer(b"ACGTNacgt", np.uint8)
    seqs = [bytes(rng.choice(al, int(rng.integers(0, 60)))).decode() for _ in range(n)]
    cig = []
    for s in seqs:
        parts, used = [], 0
        while used < len(s):
            op = "MIDNSHP=X"[int(rng.integers(9))]
            k = int(rng.integers(0, 8))
            parts.append(f"{k}{op}")
            used += k if op in "MIS=X" else 0
        cig.append("".join(parts))
    seqs[3] = None
    cig[4] = None
    alleles = [f"AC[{int(rng.integers(0, 40))}:{int(rng.integers(1, 4))}I]GG[None]" for _ in range(n)]
    quals = [bytes(rng.integers(33, 74, int(rng.integers(0, 30)), dtype=np.uint8)).decode() for _ in range(n)]
    quals[7] = None
    for lay in ("view", "utf8", "large", "chunked_view", "sliced_view", "sliced_utf8"):
        S, C, A, Q = (_layouts(v)[lay] for v in (seqs, cig, alleles, quals))
        got = plugin.call_plugin("reverse_complement_series", [S]).combine_chunks().to_pylist()
        assert got == O.column("revcomp", [seqs]), lay
        for bd in (False, True):
            got = plugin.call_plugin("parse_cigar_series", [C], {"block_dels": bd}).combine_chunks().to_pylist()
            assert got == O.column("parse_cigar", [cig], int(bd)), lay
        for name, op in (("cigar_aligned_ref_expr", "aligned_ref"), ("cigar_aligned_query_expr", "aligned_query")):
            got = plugin.call_plugin(name, [S, S, C]).combine_chunks().to_pylist()
            assert got == O.column(op, [seqs, seqs, cig]), (lay, name)
        got = plugin.call_plugin("extract_cigar_insertions_expr", [S, C]).combine_chunks().to_pylist()
        assert got == O.column("cigar_insertions", [seqs, cig]), lay
        got = plugin.call_plugin("enrich_allele_insertions_expr", [A, S, C]).combine_chunks().to_pylist()
        assert got == O.column("enrich", [alleles, seqs, cig]), lay
        got = plugin.call_plugin("phred_to_numeric_series_str", [Q], {"base": 33}).combine_chunks().to_pylist()
        assert got == O.column("phred_str", [quals], 33), lay
        got = plugin.call_plugin("phred_to_numeric_series", [Q], {"base": 33}).combine_chunks().to_pylist()
        assert got == [v for v in O.column("phred_list", [quals], 33) if v is not None], lay
    # scalar reference (pl.lit(ref)) broadcast over the query column
    ref1 = pa.array(["ACGTACGTAAcc"], type=pa.string_view())
    got = plugin.call_plugin("cigar_aligned_ref_expr", [ref1, _layouts(seqs)["view"], _layouts(cig)["view"]])
    assert got.combine_chunks().to_pylist() == O.column("aligned_ref", [["ACGTACGTAAcc"], seqs, cig])
    # serde errors: required kwargs
    assert "missing field `block_dels`" in _err("parse_cigar_series", [_layouts(cig)["view"]], {})
    assert "missing field `base`" in _err("phred_to_numeric_series_str", [_layouts(quals)["view"]], {})
