"""Helpers shared by the --reference-fasta tests: a read's own reference segment (its bases on
M / = / X with the MD mismatches substituted, MD deletions on D) and a contig-wide FASTA assembled
from the reads' segments."""
from typing import Dict, Optional

import numpy as np

from guacamole_amd.reads import ReadSet
from guacamole_amd.soa import md_events


def own_reference(rs: ReadSet, i: int) -> Optional[np.ndarray]:
    """The reference bases [start, end) a read's MD describes (None: no MD, or an N gap)."""
    if rs.md_len[i] < 0:
        return None
    co, nc = int(rs.cigar_off[i]), int(rs.n_cigar[i])
    ops = [(int(c) & 15, int(c) >> 4) for c in rs.cigar[co:co + nc]]
    if any(op == 3 for op, _ in ops):
        return None
    md = rs.md[int(rs.md_off[i]):int(rs.md_off[i]) + int(rs.md_len[i])].tobytes()
    ev, _ = md_events(md, int(rs.start[i]), ops)
    evd: Dict[int, int] = {e >> 8: e & 0xFF for e in ev}
    so = int(rs.seq_off[i])
    seq = rs.seq[so:so + int(rs.seq_len[i])]
    out = []
    rp = fp = 0
    for op, ln in ops:
        if op in (0, 7, 8):
            for j in range(ln):
                out.append(evd.get(fp + j, int(seq[rp + j])))
            rp += ln
            fp += ln
        elif op == 2:
            for j in range(ln):
                out.append(evd.get(fp + j, ord("N")))
            fp += ln
        elif op in (1, 4):
            rp += ln
    return np.array(out, np.uint8)


def assembled_reference(*read_sets: ReadSet, modify_every: int = 0, seed: int = 7) -> Dict[str, np.ndarray]:
    """Per contig: 'N' everywhere, each read's own segment written over it (later reads win), and
    with `modify_every` > 0 every k-th covered locus changed to another base."""
    rs0 = read_sets[0]
    ref = {name: np.full(int(ln), ord("N"), np.uint8) for name, ln in zip(rs0.contig_names, rs0.contig_lengths)}
    covered = {name: np.zeros(int(ln), bool) for name, ln in zip(rs0.contig_names, rs0.contig_lengths)}
    for rs in read_sets:
        for i in range(rs.n):
            seg = own_reference(rs, i)
            if seg is None:
                continue
            name = rs.contig_names[int(rs.contig[i])]
            s = int(rs.start[i])
            ref[name][s:s + len(seg)] = seg
            covered[name][s:s + len(seg)] = True
    if modify_every > 0:
        rng = np.random.default_rng(seed)
        for name in ref:
            idx = np.flatnonzero(covered[name])[::modify_every]
            alt = np.frombuffer(b"ACGT", np.uint8)
            for l in idx:
                choices = alt[alt != ref[name][l]]
                ref[name][l] = choices[rng.integers(len(choices))]
    return ref
