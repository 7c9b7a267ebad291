"""rogtk_amd — MI355X-native (gfx950) engine for rogtk's UMI score + cluster hot path.

Drop-in surface (mirrors rogtk/__init__.py's `umi` / `hamming` namespaces):

    import rogtk_amd as rg
    rg.col(umis).umi.complexity_all()            # Struct of 7 (umi_score.rs)
    rg.col(umis).umi.shannon_entropy()           # ... and the other 6 fields
    rg.col(umis).hamming.distance("ACGTACGTACGT")
    rg.col(umis).hamming.within("ACGTACGTACGT", max_distance=1)
    rg.umi_complexity_scores(umis)
    rg.umi_cluster(umis, max_distance=1)         # H3 (caller-side group_by('umi'))
    rg.kmer_spectrum(reads, k=17, min_coverage=20, group_offsets=...)  # H4 (fracture.rs)
    rg.assemble_sequences(group_reads, k=13, min_coverage=1, method="compression")  # H5
    rg.assemble_column_groups(offsets, values, cluster_ids, k=10, min_coverage=5)  # H5, all groups
    rg.col(seqs).dna.reverse_complement(); rg.parse_cigar(cigars, block_dels=False)
    rg.col(ref).cigar.align_to_ref(query, cigars); rg.extract_cigar_insertions(seq, cigars)

Device-resident pipeline (packed SoA in HBM, torch tensors as plumbing):
    rogtk_amd.device (PackedBatch, score_packed, ClusterEngine, cluster_batch)
Multi-GPU exchange: rogtk_amd.dist. Synthetic data: rogtk_amd.synth.
C ABI: include/rogtk_hip.h (librogtk_hip.so, in-tree).
"""
from ._lib import RogtkError, device_count, version  # noqa: F401
from .fastq import iter_paired_fastqs, parse_paired_fastqs  # noqa: F401
from .assembly import (  # noqa: F401
    assemble_column_groups,
    assemble_groups,
    assemble_sequences,
    assemble_sequences_with_anchors,
    optimize_assembly,
    sweep_assembly_params,
)
from .strings import (  # noqa: F401
    CigarNamespace,
    DnaNamespace,
    extract_cigar_insertions,
    parse_cigar,
    phred_to_numeric,
    phred_to_numeric_str,
    reverse_complement,
)
from .api import (  # noqa: F401
    FIELDS,
    KMER_STATS,
    STRUCT_TYPE,
    Col,
    HammingExpr,
    UmiNamespace,
    col,
    hamming_distance,
    hamming_within,
    kmer_spectrum,
    umi_cluster,
    umi_complexity,
    umi_complexity_scores,
)

__all__ = [
    "RogtkError", "device_count", "version", "FIELDS", "STRUCT_TYPE", "Col", "HammingExpr",
    "UmiNamespace", "col", "hamming_distance", "hamming_within", "umi_cluster", "umi_complexity",
    "umi_complexity_scores", "kmer_spectrum", "KMER_STATS", "assemble_sequences",
    "assemble_sequences_with_anchors", "sweep_assembly_params", "optimize_assembly", "assemble_groups",
    "assemble_column_groups", "iter_paired_fastqs",
    "parse_paired_fastqs", "DnaNamespace", "CigarNamespace", "reverse_complement", "parse_cigar",
    "phred_to_numeric_str", "phred_to_numeric", "extract_cigar_insertions",
]
