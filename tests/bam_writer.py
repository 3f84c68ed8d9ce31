"""Minimal BAM writer for ingest tests (SAM/BAM specification: BGZF blocks of raw deflate
with the BC extra subfield, then the binary header and alignment records)."""
import struct
import zlib

_SEQ = "=ACMGRSVTWYHKDBN"
_OPS = "MIDNSHP=X"


def cigar_ops(s):
    out, num = [], ""
    for ch in s:
        if ch.isdigit():
            num += ch
        else:
            out.append((int(num) << 4) | _OPS.index(ch))
            num = ""
    return out


def tag_z(tag, val):
    return tag.encode() + b"Z" + val.encode() + b"\0"


def tag_i(tag, val):
    return tag.encode() + b"i" + struct.pack("<i", val)


def tag_b(tag, sub, vals):
    fmt = {"c": "b", "C": "B", "s": "h", "S": "H", "i": "i", "I": "I", "f": "f"}[sub]
    return tag.encode() + b"B" + sub.encode() + struct.pack("<i", len(vals)) + struct.pack("<%d%s" % (len(vals), fmt),
                                                                                             *vals)


def record(ref_id, pos, name, cigar, seq, qual=None, mapq=60, flag=0, tags=b""):
    ops = (cigar_ops(cigar) if cigar != "*" else []) if isinstance(cigar, str) else list(cigar)
    l_seq = len(seq)
    packed = bytearray((l_seq + 1) // 2)
    for i, ch in enumerate(seq):
        packed[i >> 1] |= _SEQ.index(ch) << (4 * (1 - (i & 1)))
    q = bytes([0xFF] * l_seq) if qual is None else bytes(qual)
    body = struct.pack("<iiBBHHHiiii", ref_id, pos, len(name) + 1, mapq, 4680, len(ops), flag, l_seq, -1, -1, 0)
    body += name.encode() + b"\0" + struct.pack("<%dI" % len(ops), *ops) + bytes(packed) + q + tags
    return struct.pack("<i", len(body)) + body


def header(text, contigs):
    t = text.encode()
    out = b"BAM\1" + struct.pack("<i", len(t)) + t + struct.pack("<i", len(contigs))
    for name, ln in contigs:
        out += struct.pack("<i", len(name) + 1) + name.encode() + b"\0" + struct.pack("<i", ln)
    return out


def bgzf(data, block=65280, level=6):
    out = []
    for i in list(range(0, len(data), block)) + [len(data)]:  # ... + the empty EOF block
        chunk = data[i:i + block]
        if i == len(data) and out and chunk:
            break
        c = zlib.compressobj(level, zlib.DEFLATED, -15)
        comp = c.compress(chunk) + c.flush()
        bsize = 18 + len(comp) + 8
        out.append(struct.pack("<BBBBIBBHBBHH", 31, 139, 8, 4, 0, 0, 255, 6, 66, 67, 2, bsize - 1) + comp +
                   struct.pack("<II", zlib.crc32(chunk) & 0xFFFFFFFF, len(chunk)))
    return b"".join(out)


def write_bam(path, text, contigs, records, block=65280, plain_gzip=False):
    data = header(text, contigs) + b"".join(records)
    with open(path, "wb") as fh:
        if plain_gzip:
            import gzip
            fh.write(gzip.compress(data))
        else:
            fh.write(bgzf(data, block))
