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


def bgzf(data, block=65280, level=6, strategy=zlib.Z_DEFAULT_STRATEGY, offsets=None):
    """BGZF blocks of `block` input bytes each (+ the empty EOF block).  offsets: a list that
    receives each block's file offset."""
    out = []
    at = 0
    for i in list(range(0, len(data), block)) + [len(data)]:  # ... + the empty EOF block
        chunk = data[i:i + block]
        if i == len(data) and out and chunk:
            break
        c = zlib.compressobj(level, zlib.DEFLATED, -15, 8, strategy)
        comp = c.compress(chunk) + c.flush()
        bsize = 18 + len(comp) + 8
        out.append(struct.pack("<BBBBIBBHBBHH", 31, 139, 8, 4, 0, 0, 255, 6, 66, 67, 2, bsize - 1) + comp +
                   struct.pack("<II", zlib.crc32(chunk) & 0xFFFFFFFF, len(chunk)))
        if offsets is not None:
            offsets.append(at)
        at += bsize
    return b"".join(out)


def reg2bin(beg, end):
    """SAM specification §5.3: the smallest bin holding [beg, end)."""
    end -= 1
    for shift, first in ((14, 4681), (17, 585), (20, 73), (23, 9), (26, 1)):
        if beg >> shift == end >> shift:
            return first + (beg >> shift)
    return 0


def bai(data, block, offsets, n_ref, rec_starts):
    """A BAI (SAM specification §5.2) for a BAM whose inflated bytes `data` were cut into blocks
    at file offsets `offsets`, each of `block` bytes (an int) or starting at the given data
    offsets (a list); rec_starts: each record's offset in `data`."""
    import bisect
    starts = block if isinstance(block, list) else [k * block for k in range(len(offsets))]

    def voff(x):
        k = bisect.bisect_right(starts, x) - 1
        return (offsets[k] << 16) | (x - starts[k])
    bins = [dict() for _ in range(n_ref)]
    lin = [[] for _ in range(n_ref)]
    for k, x in enumerate(rec_starts):
        ref, pos = struct.unpack_from("<ii", data, x + 4)
        if ref < 0 or pos < 0:
            continue
        l_name, = struct.unpack_from("<B", data, x + 12)
        n_cig, = struct.unpack_from("<H", data, x + 16)
        span = sum(op >> 4 for op in struct.unpack_from("<%dI" % n_cig, data, x + 36 + l_name)
                   if (op & 15) in (0, 2, 3, 7, 8))
        end = pos + max(1, span)
        b, e = voff(x), voff(rec_starts[k + 1]) if k + 1 < len(rec_starts) else voff(len(data))
        ch = bins[ref].setdefault(reg2bin(pos, end), [])
        if ch and ch[-1][1] == b:
            ch[-1][1] = e
        else:
            ch.append([b, e])
        li = lin[ref]
        for w in range(pos >> 14, ((end - 1) >> 14) + 1):
            while len(li) <= w:
                li.append(0)
            if li[w] == 0 or b < li[w]:
                li[w] = b
    out = b"BAI\1" + struct.pack("<i", n_ref)
    for r in range(n_ref):
        out += struct.pack("<i", len(bins[r]))
        for bn in sorted(bins[r]):
            out += struct.pack("<Ii", bn, len(bins[r][bn])) + b"".join(struct.pack("<QQ", *c) for c in bins[r][bn])
        li = lin[r]
        for w in range(1, len(li)):  # htslib fills an empty window with the one before
            if li[w] == 0:
                li[w] = li[w - 1]
        out += struct.pack("<i", len(li)) + b"".join(struct.pack("<Q", v) for v in li)
    return out


def write_bam(path, text, contigs, records, block=65280, plain_gzip=False, level=6, strategy=zlib.Z_DEFAULT_STRATEGY,
              index=False):
    """index: also write path + ".bai"."""
    hdr = header(text, contigs)
    data = hdr + b"".join(records)
    offsets = []
    with open(path, "wb") as fh:
        if plain_gzip:
            import gzip
            fh.write(gzip.compress(data))
        else:
            fh.write(bgzf(data, block, level, strategy, offsets))
    if index:
        starts, x = [], len(hdr)
        for r in records:
            starts.append(x)
            x += len(r)
        with open(path + ".bai", "wb") as fh:
            fh.write(bai(data, block, offsets, len(contigs), starts))


def index_bam(path):
    """Write path + ".bai" for an existing BGZF BAM (any block sizes)."""
    raw = open(path, "rb").read()
    offsets, starts, parts, at, x = [], [], [], 0, 0
    while at < len(raw):
        bsize = struct.unpack_from("<H", raw, at + 16)[0] + 1
        chunk = zlib.decompress(raw[at + 18:at + bsize - 8], -15)
        offsets.append(at)
        starts.append(x)
        parts.append(chunk)
        x += len(chunk)
        at += bsize
    data = b"".join(parts)
    l_text, = struct.unpack_from("<i", data, 4)
    o = 8 + l_text
    n_ref, = struct.unpack_from("<i", data, o)
    o += 4
    for _ in range(n_ref):
        l_name, = struct.unpack_from("<i", data, o)
        o += 4 + l_name + 4
    recs = []
    while o < len(data):
        recs.append(o)
        o += 4 + struct.unpack_from("<i", data, o)[0]
    with open(path + ".bai", "wb") as fh:
        fh.write(bai(data, starts, offsets, n_ref, recs))
