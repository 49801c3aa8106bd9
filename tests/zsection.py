"""The sequences-section shape of a one-block Zstandard frame (test infrastructure only): where
zstd_fast.hip phase A' (zs_fse_parse_kernel) puts its LDS window limits.  RFC 8878 3.1.1 (frame
header), 3.1.1.2 (block header), 3.1.1.3.1 (literals section header), 3.1.1.3.2.1 (sequences
section header) and 4.1.1 (FSE table description); the table descriptions are parsed as
FSE_readNCount reads them (oracle/zstd.h zs_ncount)."""


def _ncount(b: bytes, p: int):
    """-> (bytes used, accuracy log) of the FSE table description at b[p:]."""
    def bits(bp, n):
        v = 0
        for i in range(n):
            q = bp + i
            byte = b[p + (q >> 3)] if p + (q >> 3) < len(b) else 0
            v |= ((byte >> (q & 7)) & 1) << i
        return v
    al = (b[p] & 15) + 5
    bp, rem, thr, nb, s, prev0 = 4, (1 << al) + 1, 1 << al, al + 1, 0, False
    while rem > 1:
        if prev0:
            n0 = s
            while True:
                v = bits(bp, 2)
                bp += 2
                n0 += v
                if v != 3:
                    break
            s = n0
            prev0 = False
        v = bits(bp, nb)
        mx = (2 * thr - 1) - rem
        if (v & (thr - 1)) < mx:
            c = v & (thr - 1)
            bp += nb - 1
        else:
            c = v & (2 * thr - 1)
            if c >= thr:
                c -= mx
            bp += nb
        c -= 1
        rem -= -c if c < 0 else c
        s += 1
        prev0 = c == 0
        while rem < thr and nb > 1:
            nb -= 1
            thr >>= 1
    return (bp + 7) // 8, al


def section_shape(f: bytes, shift: int):
    """For a frame at input alignment `shift` (its address mod 16) holding one compressed block with
    raw or RLE literals: dict(nseq, modes, logs, hdr = the sequences section's header bytes,
    chunks_from_section / chunks_from_bitstream = the 16-byte chunks its bytes through the
    checksum span from the chunk holding the section's / the bitstream's first byte), else None."""
    if f[:4] != b"\x28\xb5\x2f\xfd":
        return None
    fhd = f[4]
    fcsf, ss, ck, did = fhd >> 6, (fhd >> 5) & 1, (fhd >> 2) & 1, fhd & 3
    p = 5 + (0 if ss else 1) + [0, 1, 2, 4][did] + [1 if ss else 0, 2, 4, 8][fcsf]
    bh = f[p] | f[p + 1] << 8 | f[p + 2] << 16
    if (bh >> 1) & 3 != 2 or not (bh & 1):
        return None
    bs, body = bh >> 3, p + 3
    b0 = f[body]
    lt, sf = b0 & 3, (b0 >> 2) & 3
    if lt > 1:
        return None
    if sf == 1:
        hs, nlit = 2, (b0 >> 4) + (f[body + 1] << 4)
    elif sf == 3:
        hs, nlit = 3, (b0 >> 4) + (f[body + 1] << 4) + (f[body + 2] << 12)
    else:
        hs, nlit = 1, b0 >> 3
    s = body + hs + (nlit if lt == 0 else 1)
    if s >= body + bs:
        return None
    c0 = f[s]
    if c0 < 128:
        nseq, sp = c0, 1
    elif c0 < 255:
        nseq, sp = ((c0 - 128) << 8) + f[s + 1], 2
    else:
        nseq, sp = f[s + 1] + (f[s + 2] << 8) + 0x7F00, 3
    if nseq == 0:
        return None
    modes = f[s + sp]
    sp += 1
    logs = []
    for m, d in zip((modes >> 6, (modes >> 4) & 3, (modes >> 2) & 3), (6, 5, 6)):
        if m == 2:
            u, a = _ncount(f, s + sp)
            sp += u
            logs.append(a)
        elif m == 1:
            sp += 1
            logs.append(0)
        elif m == 0:
            logs.append(d)
        else:
            logs.append(-1)
    end = body + bs + (4 if ck else 0)
    last_chunk = (shift + end + 15) >> 4
    return dict(nseq=nseq, modes=modes, logs=tuple(logs), hdr=sp,
                chunks_from_section=last_chunk - ((shift + s) >> 4),
                chunks_from_bitstream=last_chunk - ((shift + s + sp) >> 4),
                hdr_end_in_chunk=((shift + s) & 15) + sp)
