"""FASTQ loader vs a plain-Python restatement of aligner.rs:107-178 (CPU)."""
import gzip
import os

import numpy as np
import pytest

from mini_parallel_amd import MswError
from mini_parallel_amd.fastq import FastqReader, count_bases_in_fastq, process_fastq_file_in_chunks


def reference_chunks(data: bytes, n: int):
    """aligner.rs:128-170 restated: BufRead::lines (strip \\n and \\r\\n), invalid
    UTF-8 lines are errors that are skipped and not counted, line % 4 == 2 is
    the sequence, chunks of n then a final partial one; >10 errors -> Err."""
    lines = data.split(b"\n")
    if lines and lines[-1] == b"":
        lines.pop()
    chunks, chunk, count, errors = [], [], 0, 0
    for raw in lines:
        if raw.endswith(b"\r"):
            raw = raw[:-1]
        try:
            s = raw.decode("utf-8")
        except UnicodeDecodeError:
            errors += 1
            if errors > 10:
                raise ValueError("too many errors")
            continue
        count += 1
        if count % 4 == 2:
            chunk.append(s)
            if len(chunk) >= n:
                chunks.append(chunk)
                chunk = []
    if chunk:
        chunks.append(chunk)
    return chunks


def write(path, data: bytes, gz: bool, members: int = 1):
    if gz:
        with open(path, "wb") as f:
            step = max(1, len(data) // members)
            for k in range(members):
                part = data[k * step:(k + 1) * step] if k < members - 1 else data[k * step:]
                f.write(gzip.compress(part))
    else:
        open(path, "wb").write(data)


def synth_fastq(n, rng, crlf=False, bad_utf8_at=(), final_newline=True):
    out = []
    for i in range(n):
        seq = bytes(rng.choice(np.frombuffer(b"ACGTN", np.uint8), int(rng.integers(0, 300))))
        rec = [b"@r%d pos=%d" % (i, i * 7), seq, b"+", b"I" * len(seq)]
        if i in bad_utf8_at:
            rec[1] = b"\xff\xfe" + seq
        out.extend(rec)
    nl = b"\r\n" if crlf else b"\n"
    data = nl.join(out)
    return data + nl if final_newline else data


@pytest.mark.parametrize("gz,members", [(False, 1), (True, 1), (True, 3)])
@pytest.mark.parametrize("crlf", [False, True])
@pytest.mark.parametrize("final_newline", [True, False])
def test_chunks_match_reference(tmp_path, gz, members, crlf, final_newline):
    rng = np.random.default_rng(1)
    data = synth_fastq(257, rng, crlf=crlf, final_newline=final_newline)
    p = str(tmp_path / ("x.fastq.gz" if gz else "x.fastq"))
    write(p, data, gz, members)
    got = []
    process_fastq_file_in_chunks(p, 50, got.append)
    assert got == reference_chunks(data, 50)
    assert count_bases_in_fastq(p) == sum(len(s) for c in got for s in c)


def test_invalid_utf8_lines_shift_phase(tmp_path):
    rng = np.random.default_rng(2)
    data = synth_fastq(40, rng, bad_utf8_at=(3, 9))
    p = str(tmp_path / "bad.fastq")
    write(p, data, False)
    got = []
    process_fastq_file_in_chunks(p, 7, got.append)
    assert got == reference_chunks(data, 7)
    with FastqReader(p) as fq:
        while len(fq.next_chunk(100, stride=512)[1]):
            pass
        assert fq.stats()["errors"] == 2


def test_too_many_errors(tmp_path):
    rng = np.random.default_rng(3)
    data = synth_fastq(30, rng, bad_utf8_at=tuple(range(11)))
    p = str(tmp_path / "worse.fastq")
    write(p, data, False)
    with pytest.raises(MswError, match="Too many read errors"):
        process_fastq_file_in_chunks(p, 5, lambda c: None)


def test_pos_tags_and_slab(tmp_path):
    rng = np.random.default_rng(4)
    data = synth_fastq(20, rng)
    p = str(tmp_path / "t.fastq.gz")
    write(p, data, True)
    with FastqReader(p) as fq:
        seqs, lens, pos = fq.next_chunk(100, stride=304, with_pos=True)
    assert list(pos) == [i * 7 for i in range(20)]
    ref = [s for c in reference_chunks(data, 100) for s in c]
    for i, s in enumerate(ref):
        assert bytes(seqs[i, :lens[i]]).decode() == s
        assert not seqs[i, lens[i]:].any()


def test_stride_too_small(tmp_path):
    p = str(tmp_path / "long.fastq")
    write(p, b"@a\n" + b"A" * 100 + b"\n+\n" + b"I" * 100 + b"\n", False)
    with FastqReader(p) as fq:
        with pytest.raises(MswError):
            fq.next_chunk(10, stride=64)


def test_missing_file():
    with pytest.raises(MswError, match="Failed to open"):
        FastqReader("/nonexistent/x.fastq.gz")


def test_empty_file(tmp_path):
    p = str(tmp_path / "e.fastq")
    write(p, b"", False)
    got = []
    process_fastq_file_in_chunks(p, 10, got.append)
    assert got == [] and count_bases_in_fastq(p) == 0


@pytest.mark.parametrize("no_libdeflate", [False, True])
@pytest.mark.parametrize("crlf", [False, True])
def test_bgzf_lane_file(tmp_path, monkeypatch, no_libdeflate, crlf):
    """Block-gzip (bgzip) lane files: inflated block by block with libdeflate
    (or by zlib with MSW_NO_LIBDEFLATE): same chunks as the restatement, with
    records split across 64 KiB block boundaries."""
    from mini_parallel_amd.synthetic import bgzf_compress
    if no_libdeflate:
        monkeypatch.setenv("MSW_NO_LIBDEFLATE", "1")
    rng = np.random.default_rng(9)
    data = synth_fastq(3000, rng, crlf=crlf)
    p = str(tmp_path / "b.fastq.gz")
    open(p, "wb").write(bgzf_compress(data))
    assert gzip.decompress(open(p, "rb").read()) == data
    got = []
    process_fastq_file_in_chunks(p, 333, got.append)
    assert got == reference_chunks(data, 333)
    assert count_bases_in_fastq(p) == sum(len(s) for c in got for s in c)
    with FastqReader(p) as fq:
        seqs, lens, pos = fq.next_chunk(5000, stride=304, with_pos=True)
    assert list(pos) == [i * 7 for i in range(3000)]


@pytest.mark.parametrize("threads", ["2", "5"])
def test_bgzf_inflate_threads(tmp_path, monkeypatch, threads):
    """MSW_INFLATE_THREADS (the CLI sets it when a file has several host CPUs):
    a file's BGZF blocks inflated by several threads give the same chunks."""
    from mini_parallel_amd.synthetic import bgzf_compress
    monkeypatch.setenv("MSW_INFLATE_THREADS", threads)
    rng = np.random.default_rng(11)
    data = synth_fastq(5000, rng)
    p = str(tmp_path / "t.fastq.gz")
    open(p, "wb").write(bgzf_compress(data, block=4096))
    got = []
    process_fastq_file_in_chunks(p, 777, got.append)
    assert got == reference_chunks(data, 777)


def test_bgzf_corrupt_block_is_an_error(tmp_path):
    from mini_parallel_amd.synthetic import bgzf_compress
    rng = np.random.default_rng(10)
    blob = bytearray(bgzf_compress(synth_fastq(2000, rng)))
    blob[70000] ^= 0xFF  # inside the second block's deflate data
    p = str(tmp_path / "c.fastq.gz")
    open(p, "wb").write(bytes(blob))
    with pytest.raises(MswError):
        process_fastq_file_in_chunks(p, 100000, lambda c: None)


@pytest.mark.parametrize("cap", [1, 64, 700, 1 << 20])
def test_packed_reader_any_length(tmp_path, cap):
    """msw_fastq_next_packed: sequences of any length (here up to 5000 bases,
    longer than any slab stride) back to back; a sequence that does not fit
    is held for the next call and reported through `need`."""
    rng = np.random.default_rng(11)
    seqs = [bytes(rng.choice(np.frombuffer(b"ACGT", np.uint8), int(k)))
            for k in rng.integers(0, 5000, 60)]
    data = b"".join(b"@r%d\n%s\n+\n%s\n" % (i, s, b"I" * len(s)) for i, s in enumerate(seqs))
    p = str(tmp_path / "long.fastq.gz")
    write(p, data, True)
    got = []
    with FastqReader(p) as fq:
        c = cap
        while True:
            buf, lens, need = fq.next_packed(7, c)
            assert int(lens.sum()) == len(buf) <= c
            ends = np.cumsum(lens.astype(np.int64))
            got += [buf[e - l:e].tobytes() for e, l in zip(ends, lens)]
            if need:
                assert need == len(seqs[len(got)]) and need > c - len(buf)
                c = max(c, need)
            elif len(lens) == 0:
                break
    assert got == seqs
    # the compat driver's chunks: exactly N reads concatenated, any length
    with FastqReader(p) as fq:
        cat, lens = fq.next_concat(25)
    assert cat.tobytes() == b"".join(seqs[:25]) and list(lens) == [len(s) for s in seqs[:25]]
    chunks = []
    process_fastq_file_in_chunks(p, 25, chunks.append)
    assert chunks == reference_chunks(data, 25)
