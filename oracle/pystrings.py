"""TEST INFRASTRUCTURE ONLY — CPU restatement of rogtk's element-wise string
expressions, the checker for rogtk_amd/csrc/strings.hip.

Pure-Python loops over Python str (the reference takes Rust &str, i.e. valid
UTF-8), written from the reference's Rust line by line. Rust release-build
arithmetic (Cargo.toml [profile.release], no overflow checks): usize wraps at
2^64, `u8 - base` wraps at 2^8.

Parity pins: the reference ships no tests for these expressions
(tests/test_rogtk.py only imports); the known answers are the docstring examples
of rogtk/__init__.py:536-660 (CigarNamespace) and expressions.rs:81-83, checked in
tests/test_strings.py. Everything else is parity by restatement.
"""
from __future__ import annotations

from typing import Dict, List, Optional, Tuple

M64 = (1 << 64) - 1


def _cigar_tokens(cigar: str):
    """The reference's `for c in cigar.chars()` tokenizer (expressions.rs:267-272):
    ASCII digits accumulate; any other char ends a token; `num_buf.parse::<usize>()`
    fails on an empty buffer or overflow and the op is skipped."""
    buf = ""
    for c in cigar:
        if "0" <= c <= "9":
            buf += c
            continue
        if buf and int(buf) <= M64:
            yield c, int(buf)
        buf = ""


def reverse_complement(dna: str) -> str:
    """reverse_complement_to_output, expressions.rs:966-977."""
    m = {"A": "T", "T": "A", "C": "G", "G": "C", "N": "N"}
    return "".join(m.get(c, c) for c in reversed(dna))


def parse_cigar(cigar: str, block_dels: bool) -> str:
    """parse_cigar_str, expressions.rs:450-486."""
    out: List[str] = []
    ref = 0
    for op, n in _cigar_tokens(cigar):
        if op == "D":
            if block_dels:
                out.append(f"D,{ref},{n}|")
            else:
                end = (ref + n) & M64
                p = ref
                while p < end:
                    out.append(f"D,{p},1|")
                    p += 1
            ref = (ref + n) & M64
        elif op == "I":
            out.append(f"I,{ref},{n}|")
        else:
            ref = (ref + n) & M64
    s = "".join(out)
    return s[:-1] if s.endswith("|") else s


def _latin1(b: int, upper: bool) -> str:
    """`(byte as char).to_ascii_{upper,lower}case()` (expressions.rs:277,311)."""
    c = chr(b)
    if b < 0x80:
        return c.upper() if upper else c.lower()
    return c


def expand_cigar_alignment(ref_seq: str, query_seq: str, cigar: str) -> Tuple[str, str]:
    """expand_cigar_alignment, expressions.rs:257-336 (byte-wise over ref and query)."""
    rb, qb = ref_seq.encode(), query_seq.encode()
    ar: List[str] = []
    aq: List[str] = []
    rp = qp = 0
    for op, n in _cigar_tokens(cigar):
        rk, qk = min(n, len(rb) - rp), min(n, len(qb) - qp)
        if op in "M=X":
            ar.extend(_latin1(b, True) for b in rb[rp:rp + rk])
            aq.extend(_latin1(b, True) for b in qb[qp:qp + qk])
            rp += rk
            qp += qk
        elif op == "I":
            ar.append("-" * n)
            aq.extend(_latin1(b, True) for b in qb[qp:qp + qk])
            qp += qk
        elif op in "DN":
            ar.extend(_latin1(b, True) for b in rb[rp:rp + rk])
            aq.append("-" * n)
            rp += rk
        elif op == "S":
            ar.append("-" * n)
            aq.extend(_latin1(b, False) for b in qb[qp:qp + qk])
            qp += qk
    return "".join(ar), "".join(aq)


def extract_insertions(seq: str, cigar: str) -> Dict[int, str]:
    """extract_insertions_from_cigar, expressions.rs:29-80 (HashMap: later inserts win)."""
    sb = seq.encode()
    ins: Dict[int, str] = {}
    sp = rp = 0
    for op, n in _cigar_tokens(cigar):
        if op in "M=X":
            sp = (sp + n) & M64
            rp = (rp + n) & M64
        elif op == "I":
            if (sp + n) & M64 <= len(sb):
                ins[rp] = sb[sp:sp + n].decode("utf-8", "replace")  # String::from_utf8_lossy
            sp = (sp + n) & M64
        elif op in "DN":
            rp = (rp + n) & M64
        elif op == "S":
            sp = (sp + n) & M64
    return ins


def cigar_insertions(seq: str, cigar: str) -> str:
    """extract_cigar_insertions_expr row body, expressions.rs:219-243."""
    ins = extract_insertions(seq, cigar)
    return "|".join(f"{p}:{s}" for p, s in sorted(ins.items()))


def _parse_usize(s: str) -> Optional[int]:
    """`str::parse::<usize>()`: optional '+', then ASCII digits, no overflow."""
    t = s[1:] if s.startswith("+") else s
    if not t or any(not ("0" <= c <= "9") for c in t):
        return None
    v = int(t)
    return v if v <= M64 else None


def enrich_allele(allele: str, insertions: Dict[int, str]) -> str:
    """enrich_allele_with_insertions, expressions.rs:84-163."""
    out: List[str] = []
    i, n = 0, len(allele)
    while i < n:
        c = allele[i]
        i += 1
        if c != "[":
            out.append(c)
            continue
        j = allele.find("]", i)
        if j < 0:
            out.append("[" + allele[i:])
            break
        content = allele[i:j]
        i = j + 1
        seq = None
        if content != "None" and ":" in content:
            pos_str, rest = content.split(":", 1)
            pos = _parse_usize(pos_str)
            if pos is not None and rest.endswith("I"):
                if pos > 0:
                    seq = insertions.get(pos - 1, insertions.get(pos))
                else:
                    seq = insertions.get(pos)
        out.append("[" + content + (":" + seq if seq is not None else "") + "]")
    return "".join(out)


def enrich_row(allele: Optional[str], seq: Optional[str], cigar: Optional[str]) -> Optional[str]:
    """enrich_allele_insertions_expr row body, expressions.rs:180-196."""
    if allele is None:
        return None
    if seq is None or cigar is None:
        return allele
    return enrich_allele(allele, extract_insertions(seq, cigar))


def phred_values(q: str, base: int) -> List[int]:
    """`phred_char as u8 - base` per char (expressions.rs:613-617), wrapping."""
    return [((ord(c) & 0xFF) - base) & 0xFF for c in q]


def phred_str(q: str, base: int) -> str:
    """split_string, expressions.rs:655-665."""
    return "|".join(str(v) for v in phred_values(q, base))


def column(op: str, cols: List[List[Optional[str]]], param: int = 0) -> List[Optional[object]]:
    """Row-wise application with the reference's null handling and broadcasting."""
    n = max(len(c) for c in cols)

    def get(c, i):
        return c[0] if len(c) == 1 else c[i]

    out: List[Optional[object]] = []
    for i in range(n):
        v = [get(c, i) for c in cols]
        if op == "revcomp":
            out.append(None if v[0] is None else reverse_complement(v[0]))
        elif op == "parse_cigar":
            out.append(None if v[0] is None else parse_cigar(v[0], bool(param)))
        elif op in ("aligned_ref", "aligned_query"):
            if any(x is None for x in v):
                out.append(None)
            else:
                r, q = expand_cigar_alignment(*v)
                out.append(r if op == "aligned_ref" else q)
        elif op == "cigar_insertions":
            out.append(None if any(x is None for x in v) else cigar_insertions(*v))
        elif op == "enrich":
            out.append(enrich_row(*v))
        elif op == "phred_str":
            out.append(None if v[0] is None else phred_str(v[0], param))
        elif op == "phred_list":
            out.append(None if v[0] is None else phred_values(v[0], param))
        else:
            raise ValueError(op)
    return out
