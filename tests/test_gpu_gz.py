"""GPU-side BGZF lane reader (msw_inflate.hip, msw_parse.hip, msw_gfastq.cpp).

Oracles: zlib (the reference implementation of RFC 1951 inflate, via Python's
zlib / gzip modules) for the inflated bytes, and the host reader
(msw_fastq.cpp, itself checked against a restatement of aligner.rs:107-178 in
tests/test_fastq.py) for the parsed reads.  Bit-exact comparisons throughout.
"""
import gzip
import os
import struct
import zlib

import numpy as np
import pytest

from mini_parallel_amd import MswError
from mini_parallel_amd.fastq import FastqReader, GpuFastqReader, bgzf_inflate
from mini_parallel_amd.synthetic import bgzf_compress

pytestmark = pytest.mark.gpu


def fib_text(n_syms: int, seed: int) -> bytes:
    """Symbol k appears fib(k) times: a skewed distribution whose Huffman code
    reaches zlib's 15-bit length limit (with Z_HUFFMAN_ONLY)."""
    f = [1, 1]
    while len(f) < n_syms:
        f.append(f[-1] + f[-2])
    data = np.concatenate([np.full(c, 33 + k, np.uint8) for k, c in enumerate(f)])
    np.random.default_rng(seed).shuffle(data)
    return data.tobytes()


def fastq_text(n: int, seed: int, qual="mixed", crlf=False) -> bytes:
    rng = np.random.default_rng(seed)
    out = []
    for i in range(n):
        m = int(rng.integers(60, 256))
        seq = bytes(rng.choice(np.frombuffer(b"ACGT", np.uint8), m))
        if qual == "mixed":
            q = bytes(rng.choice(np.frombuffer(b"#,:F", np.uint8), m, p=[0.02, 0.08, 0.2, 0.7]))
        else:
            q = b"I" * m
        out.append(b"@SYN:%d:%d pos=%d\n%s\n+\n%s\n" % (i // 1000, i, int(rng.integers(0, 1 << 30)), seq, q))
    t = b"".join(out)
    return t.replace(b"\n", b"\r\n") if crlf else t


def payloads():
    rng = np.random.default_rng(7)
    rnd = rng.integers(0, 256, 300_000, dtype=np.uint8).tobytes()
    chunk = rng.integers(0, 256, 5000, dtype=np.uint8).tobytes()
    periodic = b"".join(bytes(rng.integers(65, 91, p, dtype=np.uint8)) * (3000 // p) for p in (1, 2, 3, 5, 17, 64, 250, 300))
    return {
        "fastq_l1": (fastq_text(3000, 1), 1, 0),
        "fastq_l6": (fastq_text(3000, 2), 6, 0),
        "fastq_l9": (fastq_text(3000, 3), 9, 0),
        "random_l6_stored": (rnd, 6, 0),
        "level0_stored": (fastq_text(500, 4), 0, 0),
        "fixed_huffman": (fastq_text(1000, 5), 6, zlib.Z_FIXED),
        "rle": (fastq_text(1000, 6), 6, zlib.Z_RLE),
        "huffman_only": (fastq_text(1000, 8), 6, zlib.Z_HUFFMAN_ONLY),
        "long_codes": (fib_text(22, 9), 6, zlib.Z_HUFFMAN_ONLY),
        "runs_258": (b"A" * 200_000 + b"AC" * 50_000, 9, 0),
        "far_matches": (chunk * 40, 9, 0),
        "periodic_overlaps": (periodic, 9, 0),
        "all_bytes": (bytes(range(256)) * 700, 6, 0),
        "empty": (b"", 6, 0),
    }


@pytest.mark.parametrize("name", list(payloads()))
def test_inflate_matches_zlib(gpu_ctx, name):
    data, level, strategy = payloads()[name]
    blob = bgzf_compress(data, level, strategy)
    assert gzip.decompress(blob) == data
    assert bgzf_inflate(gpu_ctx, blob) == data


def test_inflate_small_members_and_fixed_tables_after_dynamic(gpu_ctx):
    # many tiny members (thousands of waves), alternating block types inside a member
    data = fastq_text(2000, 11)
    blob = bgzf_compress(data, 6, 0, block=700)
    assert bgzf_inflate(gpu_ctx, blob) == data
    # one member whose deflate stream mixes block types: a long dynamic block,
    # short flushed blocks (zlib emits them with the fixed code), incompressible
    # bytes (stored), and the empty stored blocks of Z_SYNC_FLUSH
    rnd = np.random.default_rng(3).integers(0, 256, 3000, dtype=np.uint8).tobytes()
    segs = [(data[:20000], zlib.Z_FULL_FLUSH), (b"AC", zlib.Z_FULL_FLUSH), (rnd, zlib.Z_SYNC_FLUSH),
            (b"GATTACA", zlib.Z_SYNC_FLUSH), (data[20000:40000], zlib.Z_FULL_FLUSH), (b"T" * 600, zlib.Z_FINISH)]
    c = zlib.compressobj(6, zlib.DEFLATED, -15)
    raw, plain = b"", b""
    for seg, fl in segs:
        raw += c.compress(seg) + c.flush(fl)
        plain += seg
    member = struct.pack("<4BIBBH2BHH", 0x1F, 0x8B, 8, 4, 0, 0, 0xFF, 6, ord("B"), ord("C"), 2, len(raw) + 25) + raw \
        + struct.pack("<II", zlib.crc32(plain) & 0xFFFFFFFF, len(plain))
    assert len(plain) <= 65536 and gzip.decompress(member) == plain
    assert bgzf_inflate(gpu_ctx, member) == plain


@pytest.mark.parametrize("block", [1, 3, 255, 256, 257, 4099])
def test_inflate_member_sizes(gpu_ctx, block):
    # every output misalignment and partial 256-byte CRC chunk; a 1-byte
    # member at output offset 0 makes the CRC's virtual front reach before the buffer
    data = fastq_text(40, 14)[: 3 * block + 7] if block > 3 else fastq_text(4, 14)[:601]
    blob = bgzf_compress(data, 6, 0, block=block)
    assert bgzf_inflate(gpu_ctx, blob) == data
    bad = bytearray(blob)
    bad[len(blob) - 28 - 8] ^= 0x80  # CRC of the last data member (the EOF block follows)
    with pytest.raises(MswError, match="incorrect data check"):
        bgzf_inflate(gpu_ctx, bytes(bad))


def test_inflate_large_many_spans(gpu_ctx):
    data = fastq_text(60_000, 12) * 2  # ~40 MB: thousands of members in one launch
    blob = bgzf_compress(data, 6)
    assert bgzf_inflate(gpu_ctx, blob) == data


def test_inflate_long_run_of_empty_members(fresh_ctx, monkeypatch):
    """members of ISIZE 0 (BGZF EOF blocks) add compressed bytes
    but no output, so a group bounded only by its output size could copy
    more compressed bytes than the pinned staging holds.  With 1 MiB groups
    (staging 5.125 MiB) 250k EOF blocks (7 MB) between data members must
    inflate in several groups, exactly as zlib reads them."""
    from mini_parallel_amd.synthetic import BGZF_EOF
    monkeypatch.setenv("MSW_GZ_GROUP_MB", "1")
    data = fastq_text(3000, 16)
    head = bgzf_compress(data[: len(data) // 2], 6, eof_block=False)
    tail = bgzf_compress(data[len(data) // 2:], 6)
    blob = head + BGZF_EOF * 250_000 + tail
    assert len(blob) > 7_000_000
    assert bgzf_inflate(fresh_ctx, blob) == data  # MSW_GZ_GROUP_MB: read when the context is made


def test_inflate_errors(gpu_ctx):
    data = fastq_text(400, 13)
    blob = bytearray(bgzf_compress(data, 6))
    # CRC trailer of the first member
    bsize = blob[16] | (blob[17] << 8)
    bad = bytearray(blob)
    bad[bsize + 1 - 8] ^= 0x01
    with pytest.raises(MswError, match="incorrect data check"):
        bgzf_inflate(gpu_ctx, bytes(bad))
    # ISIZE larger than the data
    bad = bytearray(blob)
    bad[bsize + 1 - 4] ^= 0x01
    with pytest.raises(MswError):
        bgzf_inflate(gpu_ctx, bytes(bad))
    # corrupted deflate bytes: some error (zlib agrees the member is bad)
    for off in (20, 40, 200, bsize - 40):
        bad = bytearray(blob)
        bad[off] ^= 0xA5
        try:
            ok = gzip.decompress(bytes(bad)) == data
        except Exception:
            ok = False
        if not ok:
            with pytest.raises(MswError):
                bgzf_inflate(gpu_ctx, bytes(bad))
    # truncated file
    with pytest.raises(MswError):
        bgzf_inflate(gpu_ctx, bytes(blob[:bsize - 5]))
    # plain gzip is not BGZF
    with pytest.raises(MswError, match="BGZF"):
        bgzf_inflate(gpu_ctx, gzip.compress(data))


# ---------------------------------------------------------------------------
# The lane reader: GPU parse == host reader, record by record
# ---------------------------------------------------------------------------
def host_reads(path, stride=256):
    seqs, lens, pos = [], [], []
    with FastqReader(path) as fq:
        while True:
            s, ln, p = fq.next_chunk(5000, stride, with_pos=True)
            if len(ln) == 0:
                break
            seqs.append(s)
            lens.append(ln)
            pos.append(p)
        st = fq.stats()
    if not seqs:
        return np.zeros((0, stride), np.uint8), np.zeros(0, np.uint16), np.zeros(0, np.int64), st
    return np.concatenate(seqs), np.concatenate(lens), np.concatenate(pos), st


def gpu_reads(ctx, path, stride=256, max_reads=3000, span=1 << 20):
    seqs, lens, pos = [], [], []
    with GpuFastqReader(ctx, path, stride, max_reads, with_pos=True, span_bytes=span) as g:
        first = 0
        while True:
            s, ln, p = g.next_batch()
            if len(ln) == 0:
                break
            seqs.append(s)
            lens.append(ln)
            pos.append(p)
            first += len(ln)
        st = g.stats()
    if not seqs:
        return np.zeros((0, stride), np.uint8), np.zeros(0, np.uint16), np.zeros(0, np.int64), st
    return np.concatenate(seqs), np.concatenate(lens), np.concatenate(pos), st


def assert_reader_parity(ctx, path, **kw):
    hs, hl, hp, hst = host_reads(path, kw.get("stride", 256))
    gs, gl, gp, gst = gpu_reads(ctx, path, **kw)
    assert len(hl) == len(gl)
    assert np.array_equal(hl, gl)
    assert np.array_equal(hp, gp)
    assert np.array_equal(hs, gs)
    assert gst["reads"] == hst["reads"] and gst["lines"] == hst["lines"] and gst["errors"] == hst["errors"]
    assert gst["bases"] == int(hl.astype(np.int64).sum())
    return len(hl)


def _reader_mode(monkeypatch, mode):
    monkeypatch.setenv("MSW_GZ_NO_MAP", "1" if mode == "copy" else "0")
    monkeypatch.setenv("MSW_GZ_IN_PLACE_MB", "0" if mode == "map_upload" else "64")


@pytest.mark.parametrize("mode", ["map", "map_upload", "copy"])
@pytest.mark.parametrize("block", [0xFF00, 1000])
@pytest.mark.parametrize("crlf", [False, True])
def test_reader_matches_host_reader(gpu_ctx, tmp_path, monkeypatch, block, crlf, mode):
    """mode "map": compressed bytes from the file's mapping (its page-cache
    pages pinned in place once, one window per span starting at the page
    boundary below the span), the file's first span read by the inflate kernel in place over
    PCIe and later spans DMA'd; "map_upload": every span DMA'd
    (MSW_GZ_IN_PLACE_MB=0); "copy": preads into pinned staging
    (MSW_GZ_NO_MAP=1)."""
    _reader_mode(monkeypatch, mode)
    data = fastq_text(20_000, 21 + block % 7, crlf=crlf)  # ~7-8 MB: several 1 MiB spans, records straddle them
    p = tmp_path / "lane.fastq.gz"
    p.write_bytes(bgzf_compress(data, 6, block=block))
    n = assert_reader_parity(gpu_ctx, str(p))
    assert n == 20_000


def _drain(g):
    seqs, lens, pos = [], [], []
    while True:
        s, ln, p = g.next_batch()
        if len(ln) == 0:
            break
        seqs.append(s)
        lens.append(ln)
        pos.append(p)
    return np.concatenate(seqs), np.concatenate(lens), np.concatenate(pos)


@pytest.mark.parametrize("mode", ["map", "copy"])
def test_reader_prefetch_next_file(gpu_ctx, tmp_path, monkeypatch, mode):
    """msw_gfastq_prefetch: the next file opened and its first window pinned
    while the current one is read; reset() to that path adopts it, reset() to
    another path (or after prefetching a missing file) opens that path as
    usual; every file reads exactly as the host reader reads it."""
    monkeypatch.setenv("MSW_GZ_NO_MAP", "1" if mode == "copy" else "0")
    files = []
    for k in range(4):
        p = tmp_path / f"lane{k}.fastq.gz"
        p.write_bytes(bgzf_compress(fastq_text(6_000 + 500 * k, 40 + k), 6))
        files.append(str(p))
    with GpuFastqReader(gpu_ctx, files[0], 256, 2500, with_pos=True, span_bytes=1 << 20) as g:
        g.prefetch(files[1])  # adopted by the next reset
        got = [_drain(g)]
        g.reset(files[1])
        g.prefetch(files[3])  # not adopted: the reset names another file
        got.append(_drain(g))
        g.reset(files[2])
        g.prefetch(str(tmp_path / "missing.fastq.gz"))  # fails in the background; harmless
        got.append(_drain(g))
        g.reset(files[3])
        got.append(_drain(g))
    for f, (gs, gl, gp) in zip(files, got):
        hs, hl, hp, _ = host_reads(f)
        assert np.array_equal(hl, gl) and np.array_equal(hp, gp) and np.array_equal(hs, gs), f


@pytest.mark.parametrize("retire", [None, "0"])
@pytest.mark.parametrize("span", [1 << 20, 1 << 18])
def test_reader_prefetch_chain(gpu_ctx, tmp_path, monkeypatch, span, retire):
    """Lane files read back to back, each with the next one prefetched (the
    --full-wgs worker's order: reset, then prefetch the file after it), so
    every file after the first is adopted with its first span indexed on the
    prefetch thread; every file reads exactly as the host reader reads it.
    A finished file stays pinned until the reader closes (default), or, with
    MSW_GZ_RETIRE_MB=0, is unpinned and unmapped on the retire thread as the
    next one opens."""
    monkeypatch.setenv("MSW_GZ_NO_MAP", "0")
    if retire is None:
        monkeypatch.delenv("MSW_GZ_RETIRE_MB", raising=False)
    else:
        monkeypatch.setenv("MSW_GZ_RETIRE_MB", retire)
    files = []
    for k in range(5):
        p = tmp_path / f"lane{k}.fastq.gz"
        p.write_bytes(bgzf_compress(fastq_text(5_000 + 700 * k, 30 + k), 6))
        files.append(str(p))
    got = []
    with GpuFastqReader(gpu_ctx, files[0], 256, 3000, with_pos=True, span_bytes=span) as g:
        for k, f in enumerate(files):
            if k:
                g.reset(f)
            if k + 1 < len(files):
                g.prefetch(files[k + 1])
            got.append(_drain(g))
    for f, (gs, gl, gp) in zip(files, got):
        hs, hl, hp, _ = host_reads(f)
        assert np.array_equal(hl, gl) and np.array_equal(hp, gp) and np.array_equal(hs, gs), f


@pytest.mark.parametrize("threads", ["3", "8"])
def test_reader_parallel_compressed_reads(gpu_ctx, tmp_path, monkeypatch, threads):
    """Compressed top-ups of 32 MiB or more split over several positioned-read
    threads (MSW_GZ_READ_THREADS), parts ending mid-member: a lane file of
    stored (level 0) BGZF members, ~35 MB, read in copied mode."""
    monkeypatch.setenv("MSW_GZ_NO_MAP", "1")
    monkeypatch.setenv("MSW_GZ_READ_THREADS", threads)
    data = fastq_text(100_000, 23)
    blob = bgzf_compress(data, 0, block=0xFF00)
    assert len(blob) >= 32 << 20
    p = tmp_path / "lane.fastq.gz"
    p.write_bytes(blob)
    assert assert_reader_parity(gpu_ctx, str(p)) == 100_000


@pytest.mark.parametrize("mode", ["map", "map_upload", "copy"])
def test_reader_edge_files(gpu_ctx, tmp_path, monkeypatch, mode):
    """Tiny and odd files; in "map" mode each is one span read in place, so
    the kernel's input loads (clamped to the span) end inside the file's last
    page."""
    _reader_mode(monkeypatch, mode)
    rng = np.random.default_rng(5)
    cases = {
        "empty": b"",
        "no_final_newline": fastq_text(50, 1)[:-1],
        "only_headers": b"@a pos=1\n",
        "seq_at_eof": b"@a pos=12\nACGT",
        "blank_lines": b"\n\n\n\n@x pos=3\nAC\n+\nII\n\n\n",
        "pos_forms": b"@q pos=x pos=-7\nA\n+\nI\n@r pos=\nC\n+\nI\n@s pos=123456789012\nG\n+\nI\n@t\nT\n+\nI\n",
        "len0_and_256": b"@a pos=1\n\n+\n\n@b pos=2\n" + b"A" * 256 + b"\n+\n" + b"I" * 256 + b"\n",
        "utf8_valid_multibyte": "@é中 pos=9\nACGT\n+\néééé\n".encode() * 20,
    }
    for name, data in cases.items():
        p = tmp_path / f"{name}.fastq.gz"
        p.write_bytes(bgzf_compress(data, 6, block=int(rng.integers(5, 200))))
        assert_reader_parity(gpu_ctx, str(p))
    # a file holding only the BGZF EOF block
    p = tmp_path / "eof_only.fastq.gz"
    p.write_bytes(bgzf_compress(b"", 6))
    assert_reader_parity(gpu_ctx, str(p))


def test_reader_invalid_utf8_lines(gpu_ctx, tmp_path):
    base = fastq_text(4000, 31).split(b"\n")
    # ten invalid lines spread over the file (<= 10: skipped, not counted)
    for k in range(10):
        i = 37 + 997 * k
        base[i] = b"\xff\xfe" + base[i]
    data = b"\n".join(base)
    p = tmp_path / "bad10.fastq.gz"
    p.write_bytes(bgzf_compress(data, 6, block=3000))
    assert_reader_parity(gpu_ctx, str(p))
    # an eleventh one fails the file, with the host reader's message
    base[3900] = b"\xc0\xaf" + base[3900]
    p2 = tmp_path / "bad11.fastq.gz"
    p2.write_bytes(bgzf_compress(b"\n".join(base), 6, block=3000))
    with pytest.raises(MswError) as eh:
        host_reads(str(p2))
    with pytest.raises(MswError) as eg:
        gpu_reads(gpu_ctx, str(p2))
    assert str(eg.value) == str(eh.value)


def test_reader_too_long_sequence(gpu_ctx, tmp_path):
    data = fastq_text(100, 41) + b"@long pos=1\n" + b"A" * 300 + b"\n+\n" + b"I" * 300 + b"\n"
    p = tmp_path / "long.fastq.gz"
    p.write_bytes(bgzf_compress(data, 6))
    with pytest.raises(MswError) as eh:
        host_reads(str(p))
    with pytest.raises(MswError) as eg:
        gpu_reads(gpu_ctx, str(p))
    assert eh.value.code == eg.value.code == -2  # MSW_E_RANGE


def test_reader_rejects_plain_gzip(gpu_ctx, tmp_path):
    p = tmp_path / "plain.fastq.gz"
    p.write_bytes(gzip.compress(fastq_text(10, 1)))
    with pytest.raises(MswError, match="BGZF"):
        GpuFastqReader(gpu_ctx, str(p))


@pytest.mark.parametrize("cut", [1, 2, 7, 40, 300])
def test_inflate_truncated_deflate_stream(gpu_ctx, cut):
    """A member whose deflate data is cut short (BSIZE, CRC and ISIZE left
    consistent with the shorter member): the decode runs into the trailer
    and the next member's bytes, which the token loop merges unchecked, and
    must still report truncation -- zlib says the stream is incomplete."""
    data = fastq_text(300, 21)[:60000]
    c = zlib.compressobj(6, zlib.DEFLATED, -15)
    cdata = c.compress(data) + c.flush()
    short = cdata[:len(cdata) - cut]
    with pytest.raises(zlib.error):
        zlib.decompress(short, -15)
    member = (struct.pack("<4BIBBH2BHH", 0x1F, 0x8B, 8, 4, 0, 0, 0xFF, 6, ord("B"), ord("C"), 2, len(short) + 25)
              + short + struct.pack("<II", zlib.crc32(data) & 0xFFFFFFFF, len(data)))
    blob = member + bgzf_compress(fastq_text(40, 22), 6)  # another member follows
    with pytest.raises(MswError, match="truncated deflate data"):
        bgzf_inflate(gpu_ctx, blob)



@pytest.mark.parametrize("stride,lo,hi", [(512, 200, 512), (5008, 1, 5000)])
def test_reader_wide_slabs(gpu_ctx, tmp_path, stride, lo, hi):
    """Slab rows wider than 256 bytes (long reads, MSW_MAX_READ_LEN): the
    emit pass writes each row 256 bytes per pass of the read's 16 lanes;
    same reads, lengths and pos= as the host reader at that stride."""
    rng = np.random.default_rng(stride)
    recs = []
    for i in range(1500):
        m = int(rng.integers(lo, hi + 1))
        seq = bytes(np.frombuffer(b"ACGTN", np.uint8)[rng.integers(0, 5, m)])
        recs.append(b"@r%d pos=%d\n" % (i, int(rng.integers(0, 10 ** 9))) + seq + b"\n+\n" + b"I" * m + b"\n")
    p = tmp_path / "wide.fastq.gz"
    p.write_bytes(bgzf_compress(b"".join(recs), 6, block=20000))
    assert assert_reader_parity(gpu_ctx, str(p), stride=stride, max_reads=700) == 1500


@pytest.mark.parametrize("max_reads,group", [(64, 1), (7, 4)])
def test_reader_batch_length_bound(gpu_ctx, tmp_path, max_reads, group):
    """Each batch's max_len (the bound the scorer picks its kernel by) is the
    longest read of its own run of batches, not of the whole span: two
    300-base reads among 20..150-base ones widen only their runs' batches.
    A run is `group` batches when a span holds more than 256 batches."""
    rng = np.random.default_rng(77)
    n, outliers = 12000, (500, 7000)
    recs = []
    for i in range(n):
        m = 300 if i in outliers else int(rng.integers(20, 151))
        seq = bytes(np.frombuffer(b"ACGT", np.uint8)[rng.integers(0, 4, m)])
        recs.append(b"@r%d\n" % i + seq + b"\n+\n" + b"I" * m + b"\n")
    p = tmp_path / "bound.fastq.gz"
    p.write_bytes(bgzf_compress(b"".join(recs), 6, block=20000))
    wide, got = 0, 0
    with GpuFastqReader(gpu_ctx, str(p), 512, max_reads, span_bytes=1 << 20) as g:
        while True:
            _, ln = g.next_batch()
            if len(ln) == 0:
                break
            d = g.last
            assert d.max_len >= int(ln.max()) and d.min_len <= int(ln.min())
            wide += d.max_len >= 300
            got += len(ln)
    assert got == n
    assert 2 <= wide <= 2 * group


def test_reader_on_the_default_stream(gpu_ctx, tmp_path):
    """the reader's stream is a blocking stream (ordered with the
    null stream).  With PyTorch work queued on its default stream between
    batches -- which then serialises with inflate and parse -- every batch
    still reads exactly as the host reader reads it."""
    import ctypes

    import torch
    from mini_parallel_amd._lib import DevReadsT, check, lib
    p = tmp_path / "lane.fastq.gz"
    p.write_bytes(bgzf_compress(fastq_text(9_000, 33), 6, block=4000))
    hs, hl, _, _ = host_reads(str(p), 256)
    dev = torch.device("cuda", 0)
    x = torch.ones(1 << 22, device=dev)
    L = lib()
    got_s, got_l = [], []
    with GpuFastqReader(gpu_ctx, str(p), 256, 1000, span_bytes=1 << 20) as g:
        while True:
            with torch.cuda.stream(torch.cuda.default_stream(dev)):
                x = x * 1.0001 + 1.0  # default-stream work in flight while the reader inflates and parses
            d = DevReadsT()
            check(L.msw_gfastq_next(g._h, None, ctypes.byref(d)))
            n = int(d.n)
            if n == 0:
                break
            check(L.msw_synchronize(gpu_ctx.handle))  # the emit ran on the context's compute stream
            s = np.zeros((n, 256), np.uint8)
            ln = np.zeros(n, np.uint16)
            check(L.msw_memcpy_d2h(gpu_ctx.handle, s.ctypes.data, d.reads, s.nbytes))
            check(L.msw_memcpy_d2h(gpu_ctx.handle, ln.ctypes.data, d.read_len, ln.nbytes))
            got_s.append(s)
            got_l.append(ln)
    assert np.array_equal(np.concatenate(got_l), hl) and np.array_equal(np.concatenate(got_s), hs)
    assert torch.isfinite(x).all()


@pytest.mark.parametrize("residue", [0, 1, 2, 3, 4093])
def test_reader_in_place_file_end_at_page_boundary(gpu_ctx, tmp_path, monkeypatch, residue):
    """A lane file read in place (its one span inflated by the kernel straight
    from the pinned page-cache pages) whose size is `residue` bytes past a
    4 KiB page boundary: the kernel's input loads are clamped to the span's
    last dword, which may straddle the file's end but never the page after
    it.  The last member's header line is padded until the size fits."""
    monkeypatch.setenv("MSW_GZ_NO_MAP", "0")
    monkeypatch.setenv("MSW_GZ_IN_PLACE_MB", "64")
    main = bgzf_compress(fastq_text(3000, 71), 6, eof_block=False)
    eof = bgzf_compress(b"", 6)  # the EOF block alone
    data = None
    for pad in range(0, 8200):
        rec = b"@pad" + b"x" * pad + b" pos=5\nACGTNACGT\n+\nIIIIIIIII\n"
        blob = main + bgzf_compress(rec, 0, eof_block=False) + eof
        if len(blob) % 4096 == residue % 4096 and len(blob) > 4096:
            data = blob
            break
    assert data is not None
    p = tmp_path / "edge.fastq.gz"
    p.write_bytes(data)
    assert os.path.getsize(p) % 4096 == residue % 4096
    assert assert_reader_parity(gpu_ctx, str(p)) == 3001
