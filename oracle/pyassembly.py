"""TEST INFRASTRUCTURE ONLY — pure-Python restatement of rogtk's graph assembly (H4.4 + H5).

Follows the reference call path per group:
  fracture.rs:188-280 assemble_sequences (auto_k, k > 64, min_length, only_largest)
  fracture.rs:323-466 assemble_with_k: preliminary graph from the valid k-mers,
      Compression -> compress_graph (debruijn 0.3.4, stranded, SimpleCompress sum),
      ShortestPath -> djfind.rs:257-304, ShortestPathAuto -> djfind.rs:466-492
  djfind.rs:78-121 convert_to_petgraph (weight -ln((cov_a + cov_b) / 2)),
      :157-247 find_shortest_path (petgraph 0.7.1 dijkstra + backtrack, eps 1e-9),
      :309-463 endpoint candidates / path score / best pair
  expressions.rs:880-955 sweep, fracture_opt.rs:120-282 optimize
The k-mer spectrum at each (k, min_coverage) comes from the k-mer oracle
(oracle/kmer_oracle.cpp: filter_kmers + CountFilter + censored exts).

Where the reference's result depends on node order (BoomHashMap2 MPHF order: not
reproducible), this restatement and the product both use ascending k-mer order:
Rust's std BinaryHeap sift order is reproduced so Dijkstra ties resolve the same
way given that node order. Those choices are "parity unpinned" against the Rust
reference; they are pinned against this restatement.
"""
from __future__ import annotations

import math
from typing import List, Optional, Sequence

from . import pyoracle as P

BASES = "ACGT"


def _estimate_k(raw: List[bytes]) -> int:
    if not raw:
        return 31
    lens = [len(x) for x in raw if len(x) > 0]
    if not lens:
        return 31
    q = (sum(lens) / len(lens)) / 3.0
    k = int(math.floor(q + 0.5))  # f64::round (q >= 0)
    k = 2 ** 64 - 1 if k == 0 else (k - 1 if k % 2 == 0 else k)  # usize wrap
    return min(max(k, 11), 63)


class Graph:
    """Valid k-mers (ascending) with censored exts and counts."""

    def __init__(self, items: Sequence[Optional[bytes]], k_eff: int, min_cov: int):
        col = P.StrCol.from_list(list(items))
        r = P.kmer_spectrum(col, k_eff, min_cov)
        self.K = k_eff
        self.seqs = [P.kmer_to_str(h, l, k_eff) for h, l in zip(r["kmer_hi"], r["kmer_lo"])]
        self.ex = [int(e) for e in r["exts"]]
        self.cov = [int(c) for c in r["counts"]]
        self.index = {s: i for i, s in enumerate(self.seqs)}
        self.nseq = int(r["stats"][0][1])

    def right(self, i):
        return [self.index[self.seqs[i][1:] + BASES[b]] for b in range(4) if (self.ex[i] >> (4 + b)) & 1]

    def left(self, i):
        return [self.index[BASES[b] + self.seqs[i][:-1]] for b in range(4) if (self.ex[i] >> b) & 1]


def compress(g: Graph) -> List[str]:
    n = len(g.seqs)
    avail = [True] * n
    out = []
    for seed in range(n):
        if not avail[seed]:
            continue
        avail[seed] = False
        lpath, rpath = [], []
        cur = seed
        while True:
            nb = g.left(cur)
            if len(nb) != 1:
                break
            nx = nb[0]
            if not avail[nx] or len(g.right(nx)) != 1:
                break
            avail[nx] = False
            lpath.append(nx)
            cur = nx
        cur = seed
        while True:
            nb = g.right(cur)
            if len(nb) != 1:
                break
            nx = nb[0]
            if not avail[nx] or len(g.left(nx)) != 1:
                break
            avail[nx] = False
            rpath.append(nx)
            cur = nx
        path = lpath[::-1] + [seed] + rpath
        s = g.seqs[path[0]] + "".join(g.seqs[v][-1] for v in path[1:])
        if len(s) >= g.K:
            out.append(s)
    return out


class PetGraph:
    def __init__(self, g: Graph):
        n = len(g.seqs)
        self.seq = g.seqs
        self.out = [[] for _ in range(n)]  # newest first (petgraph edge lists)
        self.inc = [[] for _ in range(n)]
        for a in range(n):
            for b in g.right(a):
                w = -math.log((g.cov[a] + g.cov[b]) / 2.0)
                self.out[a].insert(0, (b, w))
                self.inc[b].insert(0, (a, w))


class RustHeap:
    """std::collections::BinaryHeap<MinScored<f64, usize>>."""

    def __init__(self):
        self.d = []

    @staticmethod
    def _le(a, b):  # a <= b in MinScored order
        return a[0] >= b[0]

    def _sift_up(self, start, pos):
        elem = self.d[pos]
        while pos > start:
            parent = (pos - 1) // 2
            if self._le(elem, self.d[parent]):
                break
            self.d[pos] = self.d[parent]
            pos = parent
        self.d[pos] = elem

    def push(self, item):
        self.d.append(item)
        self._sift_up(0, len(self.d) - 1)

    def pop(self):
        item = self.d.pop()
        if self.d:
            item, self.d[0] = self.d[0], item
            end = len(self.d)
            pos, child = 0, 1
            elem = self.d[0]
            while end >= 2 and child <= end - 2:
                child += 1 if self._le(self.d[child], self.d[child + 1]) else 0
                self.d[pos] = self.d[child]
                pos = child
                child = 2 * pos + 1
            if child == end - 1:
                self.d[pos] = self.d[child]
                pos = child
            self.d[pos] = elem
            self._sift_up(0, pos)
        return item


def dijkstra(pg: PetGraph, start: int):
    scores = {start: 0.0}
    visited = set()
    h = RustHeap()
    h.push((0.0, start))
    while h.d:
        score, node = h.pop()
        if node in visited:
            continue
        for nxt, w in pg.out[node]:
            if nxt in visited:
                continue
            ns = score + w
            if nxt in scores:
                if ns < scores[nxt]:
                    scores[nxt] = ns
                    h.push((ns, nxt))
            else:
                scores[nxt] = ns
                h.push((ns, nxt))
        visited.add(node)
    return scores


def shortest_path(pg: PetGraph, starts, ends):
    best = None
    min_total = math.inf
    for s in starts:
        dist = dijkstra(pg, s)
        for e in ends:
            if e not in dist:
                continue
            total = dist[e]
            if not total < min_total:
                continue
            path, cur, valid, it = [e], e, False, 0
            while cur != s:
                it += 1
                if it > 1000:
                    break
                best_prev, best_d = None, math.inf
                for nb, w in pg.inc[cur]:
                    if nb not in dist:
                        continue
                    ew = next(w2 for t2, w2 in pg.out[nb] if t2 == cur)
                    if abs(dist[nb] + ew - dist[cur]) < 1e-9 and dist[nb] < best_d:
                        best_d, best_prev = dist[nb], nb
                if best_prev is None:
                    break
                path.append(best_prev)
                cur = best_prev
                if cur == s:
                    valid = True
            if valid:
                path.reverse()
                best = (path, total)
                min_total = total
    return best


def _concat(pg, path, K):
    return pg.seq[path[0]] + "".join(pg.seq[v][K - 1:] for v in path[1:])


def path_assembly(g: Graph, pg: PetGraph, sa: str, ea: str) -> Optional[str]:
    starts = [i for i, s in enumerate(pg.seq) if s.startswith(sa)]
    ends = [i for i, s in enumerate(pg.seq) if s.endswith(ea)]
    if not starts or not ends:
        return None
    r = shortest_path(pg, starts, ends)
    return None if r is None else _concat(pg, r[0], g.K)


def auto_path_assembly(g: Graph, pg: PetGraph) -> Optional[str]:
    n = len(g.seqs)
    avg = (sum(g.cov) / n) if n else float("nan")
    thr_f = avg * 0.1
    thr_f = 1.0 if (thr_f != thr_f or thr_f < 1.0) else thr_f  # f64::max ignores NaN
    thr = min(65535, int(math.floor(thr_f)))
    sc = [i for i in range(n) if g.cov[i] >= thr and not pg.inc[i] and pg.out[i]]
    ec = [i for i in range(n) if g.cov[i] >= thr and not pg.out[i] and pg.inc[i]]
    if not sc or not ec:
        return None
    if len(sc) == 1 and len(ec) == 1:
        return path_assembly(g, pg, pg.seq[sc[0]], pg.seq[ec[0]])
    evaluated, best, best_score = 0, None, None
    for s in sc:
        for e in ec:
            if evaluated >= 100:
                break
            evaluated += 1
            r = shortest_path(pg, [s], [e])
            if r is None:
                continue
            path, w = r
            plen = float(sum(len(pg.seq[v]) for v in path))
            mean_cov = (1.0 / (w / len(path))) if w != 0 else math.inf
            score = 0.6 * min(plen / 5000.0, 1.0) + 0.4 * min(mean_cov / 100.0, 1.0)
            if best is None or score > best_score:
                best, best_score = _concat(pg, path, g.K), score
    return best


def assemble(items: Sequence[Optional[bytes]], k: int, min_cov: int, method: str, start_anchor=None,
             end_anchor=None, only_largest=True, min_length=None, auto_k=False) -> List[str]:
    raw = [bytes(x) for x in items if x is not None]
    if auto_k:
        k = _estimate_k(raw)
    if k > 64:
        return []
    g = Graph(items, P.effective_k(k), min_cov)
    if g.nseq == 0:
        return []
    if method == "compression":
        cs = compress(g)
    else:
        pg = PetGraph(g)
        c = path_assembly(g, pg, start_anchor, end_anchor) if method == "shortest_path" else auto_path_assembly(g, pg)
        cs = [] if c is None else [c]
    cs = [c for c in cs if len(c) >= (min_length or 0)]
    if not cs or not only_largest:
        return cs
    best = 0
    for i in range(1, len(cs)):
        if len(cs[i]) >= len(cs[best]):  # max_by_key keeps the last maximum
            best = i
    return [cs[best]]


def sweep(items, k_start, k_end, k_step, cov_start, cov_end, cov_step, method, start_anchor=None, end_anchor=None):
    rows = []
    for k in range(k_start, k_end + 1, k_step):
        for c in range(cov_start, cov_end + 1, cov_step):
            cs = assemble(items, k, c, method, start_anchor, end_anchor, True, None, False)
            rows.append((k, c, len(cs[0]) if cs else 0))
    return rows


def optimize(items, method, start_anchor, end_anchor, start_k, start_min_cov, max_iterations=50, explore_k=False,
             prioritize_length=False):
    nin = sum(1 for x in items if x is not None)

    def run(k, c):
        cs = assemble(items, k, c, method, start_anchor, end_anchor, True, None, False)
        contig = cs[0] if cs else ""
        return {"contig": contig, "k": k, "min_coverage": c, "length": len(contig),
                "anchors": start_anchor in contig and end_anchor in contig}

    tested = {(start_k, start_min_cov)}
    cur = run(start_k, start_min_cov)
    best_anch = cur if cur["anchors"] else None
    best_len = cur
    paths = [(start_k, start_min_cov, cur["length"], 0)]
    dirs = [(0, -1), (0, 1), (-1, 0), (1, 0)] if explore_k else [(0, -1), (0, 1)]
    result = None
    for _ in range(max_iterations):
        new = []
        for (pk, pc, plen, psteps) in paths:
            for dk, dc in dirs:
                k, c = pk + dk, pc + dc
                if dc == -1 and pc <= 1:
                    continue
                if dk == -1 and pk <= 4:
                    continue
                if dk == 1 and pk >= 64:
                    continue
                if (k, c) in tested:
                    continue
                tested.add((k, c))
                r = run(k, c)
                if r["anchors"] and (best_anch is None or r["length"] > best_anch["length"]):
                    best_anch = r
                if r["length"] > best_len["length"]:
                    best_len = r
                if r["anchors"] and not prioritize_length:
                    result = r
                    break
                if r["contig"]:
                    new.append((k, c, r["length"], 0 if r["length"] > plen else psteps + 1))
            if result is not None:
                break
        if result is not None or not new:
            break
        new.sort(key=lambda t: (-t[2], t[3]))  # stable
        paths = new[:4]
    if result is None:
        result = best_len if prioritize_length else best_anch
    if result is None:
        return {"contig": "", "k": 0, "min_coverage": 0, "length": 0, "input_sequences": nin}
    return {"contig": result["contig"], "k": result["k"], "min_coverage": result["min_coverage"],
            "length": result["length"], "input_sequences": nin}
