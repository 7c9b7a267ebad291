/*
 * rogtk_hip.h — C ABI of librogtk_hip.so, the MI355X-native (gfx950) engine for
 * rogtk's UMI score + cluster hot path.
 *
 * Boundary. In the reference (tzeitim/rogtk) this path is reached through polars
 * plugin calls into Rust (pyo3-polars #[polars_expr]); the per-row loops live in
 *   src/expressions.rs:1234-1284   umi_complexity_all_expr      (H1, struct of 7)
 *   src/expressions.rs:1286-1410   umi_*_expr single fields     (H1, 7 exprs)
 *   src/expressions.rs:1048-1073   hamming_distance_expr        (H2)
 *   src/expressions.rs:1075-1101   hamming_within_expr          (H2)
 *   src/umi_score.rs:17-200        calculate_umi_complexity     (H1 arithmetic)
 *   rogtk/__init__.py:206-214      caller-side group_by('umi')  (H3 semantics)
 * Each entry point below cites the reference interface it replaces. The plain-C
 * signatures (pointers + sizes, no torch / no HIP types) are what a Rust
 * `extern "C"` block, cgo, JNI or ctypes binds.
 *
 * Conventions
 *  - Every function returns ROGTK_OK (0) or an error code; the message of the
 *    last failure on the calling thread is rogtk_last_error(). No C++ exception
 *    and no abort ever crosses this boundary.
 *  - Strings use the Arrow C Data layout: offsets (int32 or int64, n+1 entries),
 *    values (UTF-8 bytes), optional validity bitmap (LSB bit order) with a bit
 *    offset. Null in -> null out (the caller reuses the input validity).
 *  - "Packed SoA": codes[i] holds a regular UMI 2 bits per base, FIRST base in the
 *    most significant bits, A=0 C=1 G=2 T=3 (code order == lexicographic order).
 *    regular_bits[i/64] bit (i%64) = row i is valid, has byte length umi_len
 *    (1..16) and contains only 'A','C','G','T'. All other valid rows are
 *    "irregular" and are computed by the byte-path kernels (same results).
 *  - Level-1 functions take DEVICE pointers and a hipStream_t passed as void*
 *    (NULL = legacy default stream); they only enqueue work (graph-capturable,
 *    no allocation, no synchronisation) unless documented otherwise.
 *  - Level-2 functions (*_host) take HOST Arrow buffers, run on a per-thread
 *    device context and return when the results are in the host buffers.
 */
#ifndef ROGTK_HIP_H
#define ROGTK_HIP_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define ROGTK_OK 0
#define ROGTK_E_INVALID 1     /* bad argument */
#define ROGTK_E_HIP 2         /* HIP runtime failure */
#define ROGTK_E_UNSUPPORTED 3 /* valid input outside what this build supports */
#define ROGTK_E_NODEVICE 4    /* no usable gfx950 device */
#define ROGTK_E_OVERFLOW 5    /* a capacity given by the caller was exceeded */

/* ------------------------------------------------------------------ basics */
const char* rogtk_version(void);
const char* rogtk_last_error(void);
/* Number of visible HIP devices (0 when none). */
int rogtk_device_count(int* out_count);
/* Pinned host memory for Arrow buffers the caller hands to the level-2 (host) entry
 * points: copies to / from it are direct DMA (pageable memory is staged through the
 * calling thread's pinned buffers). Blocks are cached for reuse after rogtk_host_free. */
int rogtk_host_alloc(size_t bytes, void** out);
int rogtk_host_free(void* p);
/* Stream-ordering events for pipelines of these kernels (plumbing, no reference
 * counterpart): never timed, and with flags & 1 released at device scope only (no
 * system-scope cache write-back at each record; host readers must synchronise the
 * stream or device instead). rogtk_event_query: *done = 1 once the event has fired. */
int rogtk_event_create(int flags, void** out);
int rogtk_event_destroy(void* ev);
int rogtk_event_record(void* ev, void* stream);
int rogtk_stream_wait_event(void* stream, void* ev);
int rogtk_event_query(void* ev, int* done);
int rogtk_event_synchronize(void* ev);
/* rogtk_event_attach_next: the next kernel this thread launches records `ev` on its own
 * dispatch packet (no marker packet on the stream); rogtk_event_attach_done: *taken = 1 if
 * one did (else the caller records it), and disarms. */
int rogtk_event_attach_next(void* ev);
int rogtk_event_attach_done(int* taken);

/*
 * Output set of UMI complexity scoring: ComplexityScore (umi_score.rs:5-13)
 * exported in the field order of umi_complexity_struct_output_type
 * (expressions.rs:1219-1232). NULL members are neither computed nor written,
 * which is how the seven single-field expressions (expressions.rs:1286-1410)
 * avoid the reference's 7x recomputation.
 */
typedef struct rogtk_umi_scores {
    double* shannon_entropy;
    double* linguistic_complexity;
    double* homopolymer_fraction;
    double* dinucleotide_entropy;
    uint32_t* longest_homopolymer_run;
    double* dust_score;
    double* combined_score;
} rogtk_umi_scores;

/* ============================ Level 1: device ============================ */

/*
 * Stage a device-resident Arrow string column into the packed SoA.
 * Writes codes[n] (0 for non-regular rows), regular_bits[ceil(n/64)], and the
 * indices of valid irregular rows to irregular_rows[0 .. *n_irregular) (order
 * unspecified; capacity n). *n_irregular is a DEVICE int64 zeroed by this call.
 * Replaces the per-row `ca.iter()` string walk of expressions.rs:1246/1054.
 */
int rogtk_stage_strings(const void* offsets, int offset_width, const uint8_t* values,
                        const uint8_t* validity, int64_t validity_offset, int64_t n,
                        int umi_len, uint32_t* codes, uint64_t* regular_bits,
                        int64_t* irregular_rows, int64_t* n_irregular, void* stream);

/*
 * Fused per-read pass over the packed SoA (the hot kernel):
 *   H1 scores   -> scores  (NULL = skip)            umi_complexity_all_expr, expressions.rs:1234
 *   H2 Hamming  -> hamming_distance[n] (u32, u32::MAX on length mismatch) and/or
 *                  hamming_within_bits[ceil(n/64)] (bit-packed Arrow boolean, LSB
 *                  order, distance <= max_distance)    expressions.rs:1048-1101
 *                  target = host bytes (any UTF-8); target == NULL skips H2
 * Rows whose regular bit is 0 get zeros everywhere (fix irregular rows up with
 * rogtk_umi_score_rows; null rows stay behind the caller's validity bitmap).
 * regular_bits == NULL means every row is regular.
 */
int rogtk_umi_score_packed(const uint32_t* codes, const uint64_t* regular_bits, int64_t n,
                           int umi_len, const rogtk_umi_scores* scores,
                           const uint8_t* target, int64_t target_len, uint32_t max_distance,
                           uint32_t* hamming_distance, uint64_t* hamming_within_bits, void* stream);

/* rogtk_umi_score_packed + rogtk_cluster_assign[_deferred] of the same rows in ONE pass
 * over the codes (cluster_ws resolved by rogtk_cluster_resolve; deferred != 0 as
 * rogtk_cluster_assign_deferred): the assign half of the H3 hot path
 * (expressions.rs:1034-1082, its per-row id lookup) fused into the H1/H2 kernel, which
 * already streams the codes. Same outputs as the two calls; falls back to them where the
 * workspace has no word labels. No presence mark (cluster_ws is the resolved workspace). */
int rogtk_umi_score_assign_packed(const uint32_t* codes, const uint64_t* regular_bits, int64_t n,
                                  int umi_len, const rogtk_umi_scores* scores, const uint8_t* target,
                                  int64_t target_len, uint32_t max_distance, uint32_t* hamming_distance,
                                  uint64_t* hamming_within_bits, const void* cluster_ws,
                                  int64_t cluster_max_distinct, uint32_t* cluster_id, int deferred,
                                  void* stream);

/*
 * Byte path: the same outputs for an explicit list of rows of a device Arrow
 * string column (rows[0 .. *n_rows_dev), at most max_rows), computed straight
 * from the UTF-8 bytes with the reference's byte semantics (umi_score.rs: every
 * byte counts toward totals; 'N'/lowercase are ordinary bytes; DUST for len>=64;
 * empty string -> combined NaN). max_len >= the byte length of every listed row
 * (sizes the entropy table). hamming_within_bits is updated with atomic OR.
 * Replaces calculate_umi_complexity (umi_score.rs:17) for non-packable UMIs.
 */
int rogtk_umi_score_rows(const void* offsets, int offset_width, const uint8_t* values,
                         const int64_t* rows, const int64_t* n_rows_dev, int64_t max_rows,
                         int64_t max_len, const rogtk_umi_scores* scores,
                         const uint8_t* target, int64_t target_len, uint32_t max_distance,
                         uint32_t* hamming_distance, uint64_t* hamming_within_bits,
                         void* stream);

/*
 * H3 — UMI cluster assignment over the packed SoA (spec: DESIGN.md §H3; the
 * reference groups in the caller, rogtk/__init__.py:206-214). Regular UMIs of
 * length umi_len (1..16) are clustered exactly (max_distance 0) or as connected
 * components of the Hamming<=1 graph (max_distance 1). Cluster ids are dense,
 * in order of each cluster's smallest code. The workspace is a device buffer of
 * rogtk_cluster_workspace_size() bytes, zeroed once by rogtk_cluster_init().
 * max_distinct bounds the distinct regular UMIs across all shards
 * (<= min(4^umi_len, total rows)).
 *
 * Single GPU:  init (once) -> mark (or score_packed with cluster_ws)
 *              -> local_bitmap -> resolve(bitmap, 1) -> assign
 * N GPUs:      each rank: mark -> local_bitmap -> all-gather the bitmaps (RCCL)
 *              -> resolve(gathered, N) -> assign. Every rank resolves the same
 *              global components, so ids are identical for any GPU count.
 */
int rogtk_cluster_workspace_size(int umi_len, int64_t max_distinct, int64_t* bytes);
int rogtk_cluster_bitmap_words(int umi_len, int64_t* words);
int rogtk_cluster_init(void* ws, int umi_len, int64_t max_distinct, void* stream);
int rogtk_cluster_mark(const uint32_t* codes, const uint64_t* regular_bits, int64_t n,
                       int umi_len, void* ws, int64_t max_distinct, void* stream);
/* presence table -> bitmap words (rogtk_cluster_bitmap_words); clears presence */
int rogtk_cluster_local_bitmap(void* ws, int umi_len, int64_t max_distinct,
                               uint64_t* bitmap_out, void* stream);
/* bitmaps: n_bitmaps bitmaps laid out back to back (all-gather output layout).
 * Enqueue-only: the global union rounds run speculatively and their convergence
 * flags are copied asynchronously to pinned host memory; rogtk_cluster_assign /
 * rogtk_cluster_stats check them (normally already complete) and finish the
 * resolve on their own stream in the rare case more rounds are needed. */
int rogtk_cluster_resolve(void* ws, int umi_len, int64_t max_distinct,
                          const uint64_t* bitmaps, int n_bitmaps, int max_distance,
                          void* stream);
/* cluster_id[i] for regular rows; 0xFFFFFFFF for the others. Completes a pending
 * resolve of this workspace first (host waits on that resolve's event). */
int rogtk_cluster_assign(const void* ws, int umi_len, int64_t max_distinct,
                         const uint32_t* codes, const uint64_t* regular_bits, int64_t n,
                         uint32_t* cluster_id, void* stream);
/* The same without the host wait: enqueues the assign right behind the resolve on
 * `stream` (the speculative rounds converge for almost every input), and remembers it.
 * rogtk_cluster_sync (or stats / rounds / the next resolve of ws) then checks the round
 * flags and, if the speculative rounds were not enough, finishes the rounds, relabels
 * and re-runs this assign on its stream. Read cluster_id only after that check. */
int rogtk_cluster_assign_deferred(const void* ws, int umi_len, int64_t max_distinct,
                                  const uint32_t* codes, const uint64_t* regular_bits, int64_t n,
                                  uint32_t* cluster_id, void* stream);
/* Completes the pending resolve of ws (and its deferred assign) on `stream`; the host
 * waits only for the resolve's flag copy. *redone (nullable) = 1 when it had to enqueue
 * more rounds + labels (+ the deferred assign) on `stream`, else 0. */
int rogtk_cluster_sync(const void* ws, void* stream, int* redone);
/* Copies {n_distinct, n_clusters, overflow, error} (int64 each) to host; syncs the stream. */
int rogtk_cluster_stats(const void* ws, int umi_len, int64_t max_distinct, int64_t* out4,
                        void* stream);
/* Diagnostics: the global hook rounds the last resolve of ws needed (completes it
 * first, like rogtk_cluster_stats); 0 when it needed none (exact mode, umi_len <= 7). */
int rogtk_cluster_rounds(const void* ws, void* stream, int* rounds);
/* Tuning / tests: hook rounds launched speculatively by rogtk_cluster_resolve
 * (1..64; 0 restores the default of 4). Process-wide. Fewer rounds never change
 * results: the rest run when assign / stats find the flags not yet converged. */
int rogtk_cluster_set_spec_rounds(int n);
/* Tests: polls a block of the single-pass rank-table scan makes on a predecessor's
 * look-back flag before it recounts its prefix from the bitmaps itself (>= 0; -1 restores
 * the default of 2^22). Process-wide. Never changes results: 0 forces the recount in
 * every block. */
int rogtk_cluster_set_lookback_polls(int n);
/* Local presence bitmap straight from the codes (7 <= umi_len <= 13), replacing
 * rogtk_cluster_mark + rogtk_cluster_local_bitmap: an 8-bit radix pass groups the codes
 * by code partition, then one workgroup per partition builds its slice of the bitmap in
 * LDS. bitmap_out: rogtk_cluster_bitmap_words() words; temp: device scratch of
 * rogtk_cluster_mark_bitmap_temp_bytes(n, umi_len) bytes. Enqueue-only. */
int rogtk_cluster_mark_bitmap_temp_bytes(int64_t n, int umi_len, int64_t* bytes);
/* Method of rogtk_cluster_mark_bitmap, process-wide (A/B knob, identical bitmaps):
 * 0 = auto (code slices in LDS for umi_len <= 12, partition sort for 13), 1 = partition
 * sort, 2 = code slices (umi_len <= 12). */
int rogtk_cluster_set_mark_method(int method);
int rogtk_cluster_mark_bitmap(const uint32_t* codes, const uint64_t* regular_bits, int64_t n, int umi_len,
                              uint64_t* bitmap_out, void* temp, int64_t temp_bytes, void* stream);
/* Round 5: rogtk_cluster_mark_bitmap in two phases on (possibly) two streams, the caller
 * ordering phase 2 after phase 1: phase 1 = the slice-bucket pass over the codes (nothing
 * when the code-slice segments do not apply to (n, umi_len)), phase 2 = the rest (slice
 * mark + merge of the chunk partials, or the partition sort); phase 0 = both (the
 * one-call form). Same temp, same bitmap. */
int rogtk_cluster_mark_bitmap_phase(const uint32_t* codes, const uint64_t* regular_bits, int64_t n, int umi_len,
                                    uint64_t* bitmap_out, void* temp, int64_t temp_bytes, int phase, void* stream);
/* Releases the host-side resolve state kept for ws (call before freeing ws). */
int rogtk_cluster_release(const void* ws);

/* ===================== sharded H3 (any umi_len 1..32) =====================
 * Device steps of rogtk_amd/dist.py umi_cluster_sharded (rogtk_amd/csrc/dist_cluster.hip):
 * the clusters of rows spread over ranks, merged with RCCL all-to-alls of distinct codes
 * and of masked-key records instead of the 4^L bitmap (the north_star's
 * "RCCL all-to-all merge"); ids identical to the single-GPU engines. Device pointers;
 * the entry points that report sizes (host int64 outputs) synchronise `stream`.
 * codes: u64 2-bit codes (first base most significant); kind: 0 null, 1 regular,
 * 2 irregular (valid, not umi_len pure ACGT). */
int rogtk_long_codes(const void* offsets, int offset_width, const uint8_t* values, const uint8_t* validity,
                     int64_t validity_offset, int64_t n, int umi_len, uint64_t* codes, uint8_t* kind,
                     void* stream);
/* Sorted distinct codes of the rows with kind 1 (kind NULL: all rows); *n_out on the host. */
int rogtk_unique_codes(const uint64_t* codes, const uint8_t* kind, int64_t n, int umi_len, uint64_t* out,
                       int64_t* n_out, void* stream);
/* Owner rank of a code = floor(code * world / 4^umi_len); counts[world] (host) of a
 * sorted array (already grouped by owner). */
int rogtk_owner_counts(const uint64_t* sorted, int64_t n, int umi_len, int world, int64_t* counts, void* stream);
/* n * umi_len records (code with digit p zeroed, p, code) of the distinct codes D, packed
 * by destination rank hash(masked code, p) % world; counts[world] (host). */
int rogtk_masked_records(const uint64_t* D, int64_t n, int umi_len, int world, uint64_t* masked, uint32_t* pos,
                         uint64_t* code, int64_t* counts, void* stream);
/* Groups received records by (p, masked code); consecutive members -> an edge between
 * their codes' indices in the global sorted distinct set G. edges: 2 x u32 per edge,
 * capacity n; *n_edges (host). */
int rogtk_clique_edges(const uint64_t* masked, const uint32_t* pos, const uint64_t* code, int64_t n, int umi_len,
                       const uint64_t* G, int64_t ng, uint32_t* edges, int64_t* n_edges, void* stream);
/* Connected components of nv vertices under m edges (2 x u32 each): labels[v] dense, in
 * order of each component's smallest vertex; *n_clusters (host). */
int rogtk_cc_labels(int64_t nv, const uint32_t* edges, int64_t m, uint32_t* labels, int64_t* n_clusters,
                    void* stream);
/* cluster_id[i] = labels[index of codes[i] in G] for kind 1, 0xFFFFFFFF for kind 0;
 * kind 2 rows untouched. Fails when a regular code is absent from G. */
int rogtk_assign_codes(const uint64_t* codes, const uint8_t* kind, int64_t n, const uint64_t* G, int64_t ng,
                       const uint32_t* labels, uint32_t* cluster_id, void* stream);
/* Exact-bytes groups of n strings (int64 offsets from 0): ids[i] = id_base + rank of the
 * string among the distinct strings in byte-lexicographic order; *n_groups (host). */
int rogtk_group_strings(const int64_t* offsets, const uint8_t* values, int64_t n, int64_t max_len, uint32_t id_base,
                        uint32_t* ids, int64_t* n_groups, void* stream);
/* Step 8 of the sharded H3 for max_distance 0 or 1: the n
 * all-gathered irregular strings (int64 offsets from 0) -> ids[n]. max_distance 0: exact
 * bytes, ids from n_reg. max_distance 1: Hamming-1 edges among the strings and to the
 * sorted global codes G[ng] (umi_len <= 32), connected components with the n_reg regular
 * clusters (labels[ng]: each G code's regular id, remapped IN PLACE when irregular strings
 * bridge regular clusters). *n_clusters = all clusters. Same result on every rank. */
int rogtk_irregular_merge(const int64_t* offsets, const uint8_t* values, int64_t n, int64_t max_len, int umi_len,
                          int max_distance, const uint64_t* G, int64_t ng, uint32_t* labels, int64_t n_reg,
                          uint32_t* ids, int64_t* n_clusters, void* stream);

/* ========================= Level 2: host buffers ========================= */

/* umi_complexity_all_expr + the 7 single-field exprs (expressions.rs:1234-1410). */
int rogtk_umi_complexity_host(const void* offsets, int offset_width, const uint8_t* values,
                              int64_t values_len, const uint8_t* validity,
                              int64_t validity_offset, int64_t n, const rogtk_umi_scores* out);

/* hamming_distance_expr / hamming_within_expr (expressions.rs:1048-1101).
 * within_bits: Arrow bit-packed (LSB order), ceil(n/8) bytes; either output NULL = skip. */
int rogtk_hamming_host(const void* offsets, int offset_width, const uint8_t* values,
                       int64_t values_len, const uint8_t* validity, int64_t validity_offset,
                       int64_t n, const uint8_t* target, int64_t target_len,
                       uint32_t max_distance, uint32_t* distance, uint8_t* within_bits);

/* H3 over a host column: regular rows clustered on the GPU (umi_len <= 0:
 * length of the first non-null row); irregular non-null rows grouped by exact
 * bytes and numbered after the regular clusters in byte-lexicographic order.
 * cluster_id of null rows = 0xFFFFFFFF. */
int rogtk_umi_cluster_host(const void* offsets, int offset_width, const uint8_t* values,
                           int64_t values_len, const uint8_t* validity, int64_t validity_offset,
                           int64_t n, int umi_len, int max_distance, uint32_t* cluster_id,
                           int64_t* n_clusters, int* resolved_umi_len);

/* H3 over a DEVICE column (int64 offsets from 0, values, optional validity bitmap at bit
 * offset 0), same semantics and ids as rogtk_umi_cluster_host; umi_len >= 1 required.
 * cluster_id is a device buffer. Enqueued on `stream`; synchronises it once (sizes). */
int rogtk_umi_cluster_dev(const int64_t* offsets, const uint8_t* values, const uint8_t* validity, int64_t n,
                          int umi_len, int max_distance, uint32_t* cluster_id, int64_t* n_clusters, void* stream);

/* ================ H4: k-mer spectra of read groups (host buffers) ================
 * Replaces, per polars group (group_by(...).agg), the k-mer front end of fracture
 * assembly: expressions.rs:739-744 (nulls skipped), fracture.rs:200-256 (auto_k via
 * estimate_k, k > 64 -> nothing, uppercase, drop sequences with a non-ACGT byte,
 * effective k = 4/8/16/32/64) and fracture.rs:105-146 (debruijn 0.3.4
 * filter_kmers + CountFilter(min_coverage) + remove_censored_exts, stranded; node /
 * terminal / isolated counts). Spec: oracle/kmer_oracle.cpp.
 * Groups are contiguous row ranges: group_offsets[0] = 0 ... group_offsets[n_groups]
 * = n_rows (NULL / 0 groups = one group of all rows).
 * Output, per group in group order (entry_offsets[n_groups + 1]): its valid k-mers
 * in ascending order (the crate's pre-MPHF order; its MPHF order is not
 * reproducible), kmers[2 i] = high 64 bits (k_eff = 64 only), kmers[2 i + 1] = low
 * 64 bits (2-bit codes, first base most significant, A0 C1 G2 T3); exts[i] = the
 * censored Exts byte (low nibble left bases, high nibble right); counts[i] =
 * occurrences (u16, saturating). group_stats[5 g ..] = {k_eff (0 when k > 64),
 * n_sequences, node_count, terminal_count, isolated_count}.
 * capacity >= rogtk_kmer_capacity() always suffices (ROGTK_E_OVERFLOW otherwise); so does
 * rogtk_kmer_capacity() / max(min_coverage, 1), since every valid k-mer takes at least
 * min_coverage observations. */
int rogtk_kmer_capacity(const void* offsets, int offset_width, int64_t n_rows, int64_t* capacity);
/* Path selection for the calling thread (default 1): groups with <= 2048 k-mer
 * observations, rows <= 2048 bases and k_eff <= 32 run entirely in LDS (one
 * wave per group for k_eff <= 16 and <= 64 rows, round 6; one workgroup per group
 * otherwise); 2: the LDS path without the wave class; 0 sends every group through
 * the global radix-sort path. Results are identical; tests use this to cover the paths. */
int rogtk_kmer_set_path(int lds_small_groups);
/* The minimizer filter (round 4; process-wide, default on, ROGTK_KMER_MZ=0 turns it off): on the
 * block path, class-3 groups whose rows all carry the repeat certificate are checked for a
 * window minimizer shared by min_coverage rows; a group without one has no valid k-mer and
 * skips the LDS kernels (kmer_kernels.hip k_minimizer_filter). Results are identical. */
int rogtk_kmer_set_filter(int minimizer_filter);
/* Device-resident form (Level 1): the column (int64 offsets, values, optional
 * validity), the optional grouping permutation rows[n_rows] (grouped row r is
 * column row rows[r]; NULL = identity) and group_offsets[n_groups + 1] over the
 * grouped rows are DEVICE buffers, as are the outputs (layout as above; kmers 2
 * words per entry). One requested k for all groups (no auto_k). Work is enqueued on
 * `stream`, but the call synchronises it: the global path sizes its buffers from
 * the data. *n_entries (host) = total entries; ROGTK_E_OVERFLOW if > capacity
 * (which rogtk_kmer_capacity over the same rows bounds). */
int rogtk_kmer_spectrum_dev(const int64_t* offsets, const uint8_t* values, const uint8_t* validity,
                            int64_t validity_offset, const int64_t* rows, int64_t n_rows,
                            const int64_t* group_offsets, int64_t n_groups, int k, int64_t min_coverage,
                            int64_t capacity, uint64_t* kmers, uint8_t* exts, uint16_t* counts,
                            int64_t* entry_offsets, int64_t* group_stats, int64_t* n_entries, void* stream);
/* A read column (int64 offsets, uint8 values, optional validity) packed once, in column
 * order, into fixed-size 2-bit blocks of block_words u64 per row (blocks: n * block_words):
 * word 0 = byte length | ACGT-clean << 32 | repeat certificate << 33 (0xFFFFFFFF for a
 * null row), then the bases, 32 per word, first base most significant. The certificate
 * (block_words 8 only) says no 16-mer at an aligned position 16 j occurs again in the row,
 * so no k-mer with k_eff 32 occurs twice; the spectrum call then skips groups of fewer
 * such rows than min_coverage (nothing valid). block_words = rogtk_read_block_words(max_len):
 * 8, 16 or 32 (rows up to 224 / 480 / 992 bases), 0 when the column is too long.
 * max_len (device int64, nullable; round 5): receives the column's longest row in bytes
 * (a per-wave reduction inside the pack kernel, zeroed on `stream` first), so a caller
 * without a bound packs at a guessed block size and repacks only when a row did not fit
 * (the spectrum call rejects rows longer than its max_len on the device as well). */
int rogtk_read_block_words(int64_t max_len);
int rogtk_pack_reads(const int64_t* offsets, const uint8_t* values, const uint8_t* validity, int64_t validity_offset,
                     int64_t n, int block_words, uint64_t* blocks, int64_t* max_len, void* stream);
/* Round 5: the longest row of a column (max of offsets[i + 1] - offsets[i], i < n) into
 * *max_len on the host (a reduction kernel on `stream` and one 8-byte read; synchronises). */
int rogtk_max_row_len(const int64_t* offsets, int64_t n, int64_t* max_len, void* stream);
/* Round 5: rogtk_kmer_spectrum_dev with the grouped rows packed straight from their ASCII
 * bytes (k_pack_gather: the 2-bit packing and the repeat certificate of rogtk_pack_reads
 * fused with the grouped staging of rogtk_kmer_spectrum_blocks; same outputs, bit-exact),
 * for columns whose rows are at most 224 bases (max_len, or < 0 to compute it over the
 * first n_column rows; ROGTK_E_UNSUPPORTED past 224). values_len: readable bytes of values. */
int rogtk_kmer_spectrum_fused(const int64_t* offsets, const uint8_t* values, int64_t values_len,
                              const uint8_t* validity, int64_t validity_offset, const int64_t* rows, int64_t n_rows,
                              const int64_t* group_offsets, int64_t n_groups, int k, int64_t min_coverage,
                              int64_t capacity, uint64_t* kmers, uint8_t* exts, uint16_t* counts,
                              int64_t* entry_offsets, int64_t* group_stats, int64_t* n_entries, int64_t max_len,
                              int64_t n_column, void* stream);
/* rogtk_kmer_spectrum_dev over a column packed by rogtk_pack_reads (same outputs,
 * bit-exact): each grouped row is staged from its block (whole 64-B lines) instead of
 * its ASCII bytes. offsets / values stay needed (capacities, the radix path). */
int rogtk_kmer_spectrum_blocks(const uint64_t* blocks, int block_words, int64_t max_len, const int64_t* offsets,
                               const uint8_t* values, const uint8_t* validity, int64_t validity_offset,
                               const int64_t* rows, int64_t n_rows, const int64_t* group_offsets, int64_t n_groups,
                               int k, int64_t min_coverage, int64_t capacity, uint64_t* kmers, uint8_t* exts,
                               uint16_t* counts, int64_t* entry_offsets, int64_t* group_stats, int64_t* n_entries,
                               void* stream);
/* polars group_by over u32 keys on the device (e.g. H3 cluster ids): rows_out[n] =
 * row indices ordered by key (stable), group_offsets_out[0 .. *n_groups] their
 * group boundaries (capacity n + 1). Synchronises the stream. */
int rogtk_group_by_key(const uint32_t* keys, int64_t n, int64_t* rows_out, int64_t* group_offsets_out,
                       int64_t* n_groups, void* stream);
/* Groups of the calling thread's last rogtk_kmer_spectrum_host call per path:
 * out2[0] = LDS path, out2[1] = global path (groups with k > 64 count in neither). */
int rogtk_kmer_path_stats(int64_t* out2);
/* Of those LDS-path groups, the ones taken off the LDS kernels by the repeat certificate
 * (round 4: every row with observations certified free of repeated aligned 16-mers by
 * rogtk_pack_reads, fewer such rows than min_coverage, k_eff 32: nothing valid). */
int rogtk_kmer_certified_groups(int64_t* out);
/* Round 5, measurement: rows of the last call's groups that the LDS kernels processed
 * (LDS-path groups not taken off by a certificate or the minimizer filter), so a caller
 * can count the k-mer observations those kernels inserted. */
int rogtk_kmer_lds_rows(int64_t* out);
/* Round 5, tests only: decisions (device, n_groups bytes; NULL / 0 turns it off) receives,
 * for each group of the next calls (indices of the call) that the minimizer filter
 * examined, 1 = emptied (no k-mer can be valid), 2 = kept, 3 = kept (too many minimizers
 * to decide); other bytes are left as they were. Calls with more groups write nothing. */
int rogtk_kmer_debug_filter(uint8_t* decisions, int64_t n_groups);
int rogtk_kmer_spectrum_host(const void* offsets, int offset_width, const uint8_t* values,
                             int64_t values_len, const uint8_t* validity, int64_t validity_offset,
                             int64_t n_rows, const int64_t* group_offsets, int64_t n_groups, int k,
                             int auto_k, int64_t min_coverage, int64_t capacity, uint64_t* kmers,
                             uint8_t* exts, uint16_t* counts, int64_t* entry_offsets,
                             int64_t* group_stats);

/* ======= H4.4 + H5: de Bruijn assembly of one read group (host C++ + GPU spectra) =======
 * One call = one polars group. The group's k-mer spectrum is computed on the GPU
 * (rogtk_kmer_spectrum_host at min_coverage 0, once per effective k per call);
 * CountFilter, censoring, graph build, compression (compress_graph, stranded,
 * summed counts) and path finding (djfind.rs: petgraph Dijkstra over -ln(mean
 * coverage) edge weights) run natively on the host. Methods: "compression",
 * "shortest_path" (start_anchor and end_anchor required), "shortest_path_auto".
 * Node order is ascending k-mer order (the reference's MPHF order is not
 * reproducible): which of several equally long contigs is "largest", and Dijkstra
 * ties, follow that order. Graph export (DOT / CSV files) is not performed. */

/* assemble_sequences_expr (expressions.rs:695-762) / assemble_sequences
 * (fracture.rs:188-280): contigs joined by '\n' into out (out_cap bytes; *out_len =
 * the full length, ROGTK_E_OVERFLOW if larger than out_cap). min_length < 0 = none.
 * Invalid method / anchor combinations fail with the reference's messages. */
int rogtk_assemble_host(const void* offsets, int offset_width, const uint8_t* values, int64_t values_len,
                        const uint8_t* validity, int64_t validity_offset, int64_t n_rows, int k,
                        int64_t min_coverage, const char* method, const char* start_anchor,
                        const char* end_anchor, int only_largest, int64_t min_length, int auto_k,
                        char* out, int64_t out_cap, int64_t* out_len, int64_t* n_contigs);

/* sweep_assembly_params_expr (expressions.rs:880-955): for k in k_start..=k_end by
 * k_step, for min_coverage in cov_start..=cov_end by cov_step: the largest contig's
 * length (0 when none). Rows in that order; *n_out rows (ROGTK_E_OVERFLOW > cap). */
int rogtk_assembly_sweep_host(const void* offsets, int offset_width, const uint8_t* values,
                              int64_t values_len, const uint8_t* validity, int64_t validity_offset,
                              int64_t n_rows, int64_t k_start, int64_t k_end, int64_t k_step,
                              int64_t cov_start, int64_t cov_end, int64_t cov_step, const char* method,
                              const char* start_anchor, const char* end_anchor, int64_t cap,
                              int64_t* out_k, int64_t* out_cov, int64_t* out_len, int64_t* n_out);

/* optimize_assembly_expr (fracture_opt.rs:120-356): greedy beam (4 paths) over
 * (k, min_coverage); out4 = {k, min_coverage, length, input_sequences} (all 0 but
 * input_sequences when no contig qualifies); the contig goes to contig. */
int rogtk_assembly_optimize_host(const void* offsets, int offset_width, const uint8_t* values,
                                 int64_t values_len, const uint8_t* validity, int64_t validity_offset,
                                 int64_t n_rows, const char* method, const char* start_anchor,
                                 const char* end_anchor, int64_t start_k, int64_t start_min_coverage,
                                 int64_t max_iterations, int explore_k, int prioritize_length, char* contig,
                                 int64_t contig_cap, int64_t* contig_len, uint32_t* out4);
/* Round 6: H5 over every group of a k-mer spectrum call at once (the C3 path's device
 * spectra copied to the host, or any rogtk_kmer_spectrum_* output at the assembly's
 * min_coverage: its entries are exactly the preliminary graph of fracture.rs:343-348, valid
 * k-mers with exts censored to valid neighbours). Assembles every group on n_threads host
 * threads (0: 16) with the method / anchors / only_largest / min_length of
 * rogtk_assemble_host and returns a result handle: per group one string, its contigs
 * joined by '\n' (expressions.rs:695-760). Groups whose stats say k_eff 0 (k > 64) or no
 * valid sequence get an empty string and 0 contigs. Replaces a per-group
 * rogtk_assemble_host call (each its own spectrum round trip) for a polars
 * group_by(...).agg(assemble_sequences) over many groups (rogtk/__init__.py:206-214). */
int rogtk_assemble_groups_host(const uint64_t* kmers, const uint8_t* exts, const uint16_t* counts,
                               const int64_t* entry_offsets, const int64_t* group_stats, int64_t n_groups,
                               const char* method, const char* start_anchor, const char* end_anchor,
                               int only_largest, int64_t min_length, int n_threads, void** result);
/* Sizes of a result (n_groups, bytes of all strings), then its contents: offsets[n_groups + 1]
 * (int64, Arrow LargeUtf8), values, n_contigs[n_groups] (each pointer nullable); free it. */
int rogtk_assembly_result_sizes(const void* result, int64_t* n_groups, int64_t* values_len);
int rogtk_assembly_result_copy(const void* result, int64_t* offsets, char* values, int64_t* n_contigs);
int rogtk_assembly_result_free(void* result);

/* ============ paired FASTQ ingest (host C++, zlib) ============
 * parse_paired_fastqs (src/lib.rs:232-428) as a streaming reader of Arrow string
 * columns: read_id, start ("0"), end ("1"), cbc, umi, cbc_qual, umi_qual, seq, qual
 * (the reference's schema, lib.rs:258-268). limit_lines < 0 = no limit (the
 * reference's `limit` counts LINES); do_rev_comp reverse-complements R2's sequence
 * and reverses its qualities. A short read (cbc_len + umi_len beyond the line) or a
 * truncated record is ROGTK_E_INVALID (a panic in the reference). */
int rogtk_fastq_pair_open(const char* r1_path, const char* r2_path, int64_t cbc_len, int64_t umi_len,
                          int64_t limit_lines, int do_rev_comp, void** reader);
/* Next batch of <= max_records records: offsets9[c] (n + 1 int64) / values9[c] for
 * the 9 columns, owned by the reader until the next call / close; *n_records = 0 at
 * the end. */
int rogtk_fastq_pair_next(void* reader, int64_t max_records, int64_t* n_records,
                          const int64_t** offsets9, const uint8_t** values9);
int rogtk_fastq_pair_close(void* reader);

/* ====== element-wise string transforms (strings.hip) ======
 * One op per reference polars expression (src/expressions.rs); null in any input the
 * reference matches on -> null out; Utf8 in, Utf8 out (PHRED_LIST: the u8 values of
 * List[UInt8], rows of null inputs are dropped by the caller as the reference does).
 * Inputs must be valid UTF-8 (Rust &str). A column of 1 row next to longer ones is
 * broadcast (the scalar reference of cigar_aligned_*_expr, expressions.rs:344-349). */
#define ROGTK_STR_REVCOMP 1          /* reverse_complement_series        :957-977           */
#define ROGTK_STR_PARSE_CIGAR 2      /* parse_cigar_series (param block_dels) :450-505      */
#define ROGTK_STR_ALIGNED_REF 3      /* cigar_aligned_ref_expr (ref, query, cigar) :257-394 */
#define ROGTK_STR_ALIGNED_QUERY 4    /* cigar_aligned_query_expr (ref, query, cigar) :396-444 */
#define ROGTK_STR_CIGAR_INSERTIONS 5 /* extract_cigar_insertions_expr (seq, cigar) :29-80,207-251 */
#define ROGTK_STR_ENRICH_ALLELE 6    /* enrich_allele_insertions_expr (allele, seq, cigar) :84-205 */
#define ROGTK_STR_PHRED_STR 7        /* phred_to_numeric_series_str (param base) :632-665   */
#define ROGTK_STR_PHRED_LIST 8       /* phred_to_numeric_series values (param base) :598-630 */

typedef struct rogtk_str_col {
    const void* offsets; /* n + 1 entries, int32 or int64 */
    int offset_width;
    const uint8_t* values;
    int64_t values_len; /* < 0: unchecked */
    const uint8_t* validity;
    int64_t validity_offset;
    int64_t n;
} rogtk_str_col;

/* Level 1 (device columns, enqueue-only): measure writes out_offsets[n_rows + 1]
 * (exclusive scan of the output byte lengths; out_offsets[n_rows] = total) and the
 * output validity (bit per row, LSB order); the caller sizes out_values from the
 * total and calls fill. temp: rogtk_str_temp_bytes(n_rows) bytes of device memory. */
int rogtk_str_temp_bytes(int64_t n_rows, int64_t* bytes);
int rogtk_str_measure(int op, const rogtk_str_col* cols, int n_cols, int64_t n_rows, int64_t param,
                      int64_t* out_offsets, uint64_t* out_valid_bits, void* temp, int64_t temp_bytes,
                      void* stream);
int rogtk_str_fill(int op, const rogtk_str_col* cols, int n_cols, int64_t n_rows, int64_t param,
                   const int64_t* offsets, uint8_t* out_values, void* stream);

/* Level 2 (host columns): the library allocates the result (malloc); free it with
 * rogtk_str_result_free. offsets are int64 (Arrow LargeUtf8), validity LSB bits. */
typedef struct rogtk_str_result {
    int64_t n;
    int64_t* offsets;
    uint8_t* values;
    int64_t values_len;
    uint8_t* validity;
    int64_t null_count;
} rogtk_str_result;
int rogtk_str_transform_host(int op, const rogtk_str_col* cols, int n_cols, int64_t n_rows, int64_t param,
                             rogtk_str_result* out);
void rogtk_str_result_free(rogtk_str_result* r);

/* ============================== profiling ================================ */
/* When enabled, every kernel launch is bracketed by HIP events on its stream. */
/* ======== multi-GPU exchange of read groups ========
 * Packs the rows of a DEVICE string column (int64 offsets from 0, values) by
 * destination rank dest[i] in [0, world) so that each destination's rows are one
 * contiguous byte range for a single all-to-all (torch.distributed / RCCL does the
 * exchange): perm[n] = rows ordered by destination (stable), packed_offsets[n + 1] /
 * packed_values (values_cap bytes; ROGTK_E_OVERFLOW beyond) the column in perm order.
 * counts[world] / byte_counts[world] are HOST arrays (rows / bytes per destination).
 * Synchronises `stream` once (the counts). */
int rogtk_route_pack(const int64_t* offsets, const uint8_t* values, const int32_t* dest, int64_t n, int world,
                     int64_t* perm, int64_t* counts, int64_t* byte_counts, int64_t* packed_offsets,
                     uint8_t* packed_values, int64_t values_cap, void* stream);

/* ============ BAM -> Arrow columns, decoded on the GPU ============
 * Host: BGZF inflate (zlib, blocks in parallel on n_threads threads, <= 0: min(16, cores))
 * and record framing. GPU: every per-record field (rogtk_amd/csrc/bam.hip). Columns
 * follow create_bam_schema (src/bam.rs:3203-3221): name, chrom, start, end, flags,
 * sequence, quality_scores; the record semantics per mode:
 *   ROGTK_BAM_NOODLES       extract_record_data_enhanced (bam.rs:170-262): "*" name ->
 *                           "unknown", 1-based start, end = start + CIGAR reference length - 1
 *   ROGTK_BAM_HTSLIB        process_htslib_records_to_batch (bam.rs:3028-3148): 1-based
 *                           start, end = start + seq_len - 1, 0xFF qualities -> null
 *   ROGTK_BAM_HTSLIB_BLOCKS process_htslib_records_to_batch (bam_htslib.rs:154-241):
 *                           0-based start, end = bam_endpos if > pos else start, IUPAC bases */
#define ROGTK_BAM_NOODLES 0
#define ROGTK_BAM_HTSLIB 1
#define ROGTK_BAM_HTSLIB_BLOCKS 2
typedef struct rogtk_bam_batch {
    /* string columns [0] name [1] chrom [2] sequence [3] quality_scores: int64 offsets
     * (n + 1, from 0), values, validity bitmap (Arrow LSB order; NULL = all valid) */
    const int64_t* offsets[4];
    const uint8_t* values[4];
    const uint8_t* validity[4];
    /* u32 columns [0] start [1] end [2] flags and their validity (NULL = all valid) */
    const uint32_t* u32[3];
    const uint8_t* u32_validity[3];
} rogtk_bam_batch;
int rogtk_bam_open(const char* path, int n_threads, void** reader);
/* One file split over workers / ranks (the reference: discover_split_points +
 * process_file_segment_with_pool, src/bam_htslib.rs:247-420, driven by
 * bam_to_arrow_ipc_htslib_bgzf_blocks :521). HOST ONLY (no GPU needed):
 *   rogtk_bam_split_points: points[0..*n_ranges] (n + 1 entries of room) = 0, BGZF block
 *     starts at or after file_size * i / n (validated: the block header and the next one),
 *     file_size; never inside the header's blocks; fewer ranges when the file is small.
 *   rogtk_bam_find_record: the bytes to skip at the start of the stream inflated from the
 *     block at c_begin before the first record that starts there: the tail of a record that
 *     straddles the split (the first offset from which 16 records, or all up to the end of
 *     the file, pass the SAMv1 structural checks).
 * rogtk_bam_open_range: a reader (as rogtk_bam_open) of the records that START in the
 *   blocks [c_begin, c_end) (c_end < 0 or past the file: to the end), after skipping
 *   `skip` bytes of the first block's stream (0 for c_begin 0, where the header is read).
 *   Its last record may run into the next range's blocks; once the range is exhausted
 *   (*n_records == 0), rogtk_bam_range_tail gives how many bytes of it lie past c_end,
 *   i.e. the next range's exact skip (-1: the range ran to the end of the file). A caller
 *   that used rogtk_bam_find_record for a range checks its skip against the previous
 *   range's tail (and re-reads the range with the tail on a mismatch). */
int rogtk_bam_split_points(const char* path, int n, int64_t* points, int* n_ranges);
int rogtk_bam_find_record(const char* path, int64_t c_begin, int64_t* skip);
int rogtk_bam_open_range(const char* path, int n_threads, int64_t c_begin, int64_t c_end, int64_t skip,
                         void** reader);
int rogtk_bam_range_tail(void* reader, int64_t* tail);
/* Binary header: reference names (lossy UTF-8) as offsets / values, and the SAM text. */
int rogtk_bam_header(void* reader, int64_t* n_ref, const int64_t** name_offsets, const uint8_t** name_values,
                     const char** text, int64_t* text_len);
/* Next <= max_records records (host buffers owned by the reader until the next call;
 * *n_records = 0 at the end). Sequence / quality columns are skipped (NULL) unless asked. */
int rogtk_bam_next(void* reader, int64_t max_records, int mode, int include_sequence, int include_quality,
                   int64_t* n_records, rogtk_bam_batch* out);
/* Same, but the batch stays in DEVICE memory (valid until the next call). The decode is
 * enqueued on `stream` without a host wait (the columns' value buffers are sized from
 * host-known bounds; rogtk_bam_check reports corrupt records); NULL: the reader's own
 * stream, synchronised before return (use a real stream for the no-sync path). */
int rogtk_bam_next_dev(void* reader, int64_t max_records, int mode, int include_sequence, int include_quality,
                       int64_t* n_records, rogtk_bam_batch* out, void* stream);
/* The UMI column of a device batch for the H1-H3 engine (config C5): source 0 = the first
 * umi_len bases of the sequence, 1 = the read name after its last `sep` byte (UMI-tools
 * READNAME_<UMI>). Device outputs: int64 offsets (n + 1), values (values_cap bytes;
 * ROGTK_E_OVERFLOW beyond), validity bitmap (ceil(n/64) u64 words). Synchronises `stream`. */
int rogtk_bam_umi_dev(const rogtk_bam_batch* batch, int64_t n, int source, int umi_len, int sep, int64_t* offsets,
                      uint8_t* values, int64_t values_cap, uint8_t* validity, void* stream);
/* The same appended to a column of several batches with NO host synchronisation (config C5
 * overlaps the host's inflate with the GPU): rows go to offsets[row_base ..] (n + 1
 * entries) and to validity bits from row_base (ORed into a zeroed bitmap), values at the
 * column's running byte count *base (a device int64, updated on the device). Rows that
 * would pass values_cap are not written and counted in *overflow (a device u64). */
int rogtk_bam_umi_append(const rogtk_bam_batch* batch, int64_t n, int source, int umi_len, int sep,
                         int64_t* offsets, uint8_t* values, int64_t values_cap, uint8_t* validity, int64_t row_base,
                         int64_t* base, unsigned long long* overflow, void* stream);
/* A device string column (offsets from 0, n + 1 entries) appended the same way. */
int rogtk_bam_append_strings(const int64_t* src_offsets, const uint8_t* src_values, int64_t n, int64_t* offsets,
                             uint8_t* values, int64_t values_cap, int64_t row_base, int64_t* base,
                             unsigned long long* overflow, void* stream);
/* Round 6: k device string columns (int64 offsets from 0, n_i + 1 entries; values; validity
 * bitmaps) concatenated in order into out_offsets (sum n_i + 1), out_values (values_cap
 * bytes; rows past it counted in *overflow, a device u64) and out_validity, with the running
 * byte count in *base (a device int64): no host synchronisation. Arrays of device pointers
 * on the host. */
int rogtk_concat_strings_dev(int k, const int64_t* const* offsets, const uint8_t* const* values,
                             const uint64_t* const* validity, const int64_t* counts, int64_t* out_offsets,
                             uint8_t* out_values, int64_t values_cap, uint64_t* out_validity, int64_t* base,
                             unsigned long long* overflow, void* stream);
/* Raw record bytes of the reader's current batch (bounds a device batch's columns: name
 * <= 3 x bytes + 7 per record, sequence / qualities <= bytes). */
int rogtk_bam_batch_bytes(void* reader, int64_t* bytes);
/* rogtk_bam_next_dev batches do not synchronise: this checks, once, that no record of
 * the device-mode batches so far overran its block_size (synchronises `stream`). */
int rogtk_bam_check(void* reader, void* stream);
int rogtk_bam_close(void* reader);
/* Diagnostics: seconds spent so far in {file read, buffer moves + block framing, BGZF
 * inflate, record framing, H2D + GPU decode, D2H of host batches}. */
int rogtk_bam_timers(void* reader, double* out6);
/* Copies bytes between any two buffers (device or host; hipMemcpyDefault) on `stream`
 * and synchronises it: lets bindings move device batch columns into their own buffers. */
int rogtk_copy(void* dst, const void* src, int64_t bytes, void* stream);

/* ============ polars plugin ABI (rogtk_amd/csrc/polars_plugin.cpp) ============
 * librogtk_hip.so also exports the symbols polars resolves for the reference's
 * register_plugin_function calls (pyo3-polars 0.17 #[polars_expr], Cargo.toml:39):
 *   void _polars_plugin_<name>(SeriesExport*, size_t, const uint8_t* kwargs, size_t,
 *                              SeriesExport* out, CallerContext*);
 *   void _polars_plugin_field_<name>(ArrowSchema*, size_t, ArrowSchema* out,
 *                                    const uint8_t* kwargs, size_t);
 *   uint32_t _polars_plugin_get_version(void);
 *   const char* _polars_plugin_get_last_error_message(void);
 * for <name> in umi_complexity_all_expr, umi_{shannon_entropy, linguistic_complexity,
 * homopolymer_fraction, dinucleotide_entropy, combined_score, longest_homopolymer,
 * dust_score}_expr (expressions.rs:1234-1410), hamming_{distance,within}_expr
 * (:1048-1101), assemble_sequences_expr (:695), assemble_sequences_with_anchors_expr
 * (:770), sweep_assembly_params_expr (:880), optimize_assembly_expr
 * (fracture_opt.rs:283). The structs are the Arrow C Data Interface and polars-ffi
 * version_0's SeriesExport {ArrowSchema* field; ArrowArray** arrays; size_t len;
 * void (*release)(SeriesExport*); void* private_data;}; see INTEGRATION.md.
 * Diagnostics: the kwargs pickle as the plugin parses it, "key=value" lines. */
int rogtk_plugin_kwargs_debug(const uint8_t* kwargs, int64_t len, char* out, int64_t cap, int64_t* out_len);

/* Launch-bracketing HIP events (on the launch stream) around the library's kernels. */
int rogtk_profile_enable(int on);
/* Restricts the bracketing to one kernel name (below) or a comma-separated list of them;
 * NULL or "" = every kernel. Each
 * bracketed launch adds two event records to its stream, so a timed region should
 * select only the kernel it reports. */
int rogtk_profile_select(const char* kernel);
int rogtk_profile_reset(void);
/* Total device milliseconds and launch count recorded for `kernel` (synchronises
 * the recorded events). Kernel names: "stage", "score_packed", "score_rows",
 * "cluster_mark", "cluster_bitmap", "cluster_scan", "cluster_compact",
 * "cluster_union", "cluster_flatten", "cluster_label", "cluster_assign", "cluster_irregular",
 * "bam_fields", "bam_scan", "bam_fill", "pack_reads", "row_gather", "kmer_lds" (the last
 * three and score_packed: events on the dispatch packet = kernel execution time). */
int rogtk_profile_read(const char* kernel, double* total_ms, int64_t* launches);
/* Kernels that support it (k_score_packed) also time their own execution span while
 * profiled: max over workgroups of the exit clock - min of the entry clock (device
 * wall clock), i.e. the duration rocprofv3's kernel trace reports, without the fences of
 * the bracketing stream events. Totals since rogtk_profile_reset. */
int rogtk_profile_read_span(const char* kernel, double* total_ms, int64_t* launches);

#ifdef __cplusplus
}
#endif
#endif /* ROGTK_HIP_H */
