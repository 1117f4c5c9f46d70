"""The host C++ under AddressSanitizer + UBSan (CPU).

`make -C mini_parallel_amd/csrc asan` builds the host translation units
(runtime, FASTQ reader, GPU lane reader driver) instrumented, the CLI and a
reader driver (tests/c/fastq_dump.cpp) as instrumented executables.  Here the
reader cases of tests/test_fastq.py run through the driver -- every chunk
checked against the restatement of aligner.rs:107-178 -- and the CPU cases of
tests/test_cli.py through the instrumented CLI.  Any sanitizer report fails
the run (UBSan is built non-recoverable; ASan aborts on the first error and
LeakSanitizer reports leaks at exit)."""
import gzip
import os
import subprocess

import numpy as np
import pytest

from test_fastq import reference_chunks, synth_fastq, write

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
ASAN = os.path.join(ROOT, "build", "asan")
DUMP = os.path.join(ASAN, "fastq_dump")
CLI = os.path.join(ASAN, "rustseq_mini")
SAN_ENV = {"ASAN_OPTIONS": "abort_on_error=0:halt_on_error=1:detect_leaks=1:exitcode=86",
           "UBSAN_OPTIONS": "print_stacktrace=1:halt_on_error=1"}


@pytest.fixture(scope="module", autouse=True)
def asan_build():
    # Built here by __graft_entry__.build(); the GPU box gets the binaries with
    # the tree (its snapshot has no kernel objects to relink from).
    if os.path.exists("/dev/kfd") and os.access(DUMP, os.X_OK) and os.access(CLI, os.X_OK):
        return
    jobs = str(min(8, os.cpu_count() or 1))
    r = subprocess.run(["make", "-C", os.path.join(ROOT, "mini_parallel_amd", "csrc"), "-j", jobs, "asan"],
                       capture_output=True, text=True)
    if r.returncode != 0 or not (os.access(DUMP, os.X_OK) and os.access(CLI, os.X_OK)):
        # the sanitizer runtime is optional tooling: say why, do not fail the suite
        pytest.skip("host ASan/UBSan variant unavailable (make asan failed): " + r.stderr[-500:])


def run(exe, args, env=None, cwd=None):
    e = dict(os.environ)
    e.update(SAN_ENV)
    e.update(env or {})
    r = subprocess.run([exe] + [str(a) for a in args], capture_output=True, env=e, cwd=cwd, timeout=120)
    err = r.stderr.decode(errors="replace")
    assert "Sanitizer" not in err and "runtime error" not in err, err[-4000:]
    assert r.returncode != 86, err[-4000:]
    return r


def dump(*args, ok=True, env=None):
    r = run(DUMP, args, env=env)
    out = r.stdout.split(b"\n")
    if ok:
        assert r.returncode == 0, r.stdout[-2000:]
    return r.returncode, [ln for ln in out if ln]


def parse_chunks(lines):
    """-> (chunks of decoded sequences, [(len, pos)] per read, stats or None)."""
    chunks, meta, stats = [], [], None
    for ln in lines:
        tag, _, rest = ln.partition(b" ")
        if tag == b"C":
            chunks.append([])
        elif tag == b"S":
            n, pos, seq = rest.split(b" ", 2) if rest.count(b" ") >= 2 else (*rest.split(b" "), b"")
            assert len(seq) == int(n)
            chunks[-1].append(seq.decode())
            meta.append((int(n), int(pos)))
        elif tag == b"T":
            stats = tuple(int(x) for x in rest.split())
        elif tag in (b"PADERR", b"SIZEERR"):
            raise AssertionError(ln)
    return [c for c in chunks if c], meta, stats


@pytest.mark.parametrize("gz,members", [(False, 1), (True, 1), (True, 3)])
@pytest.mark.parametrize("crlf", [False, True])
@pytest.mark.parametrize("final_newline", [True, False])
def test_chunks_match_reference(tmp_path, gz, members, crlf, final_newline):
    rng = np.random.default_rng(1)
    data = synth_fastq(257, rng, crlf=crlf, final_newline=final_newline)
    p = str(tmp_path / ("x.fastq.gz" if gz else "x.fastq"))
    write(p, data, gz, members)
    got, _, _ = parse_chunks(dump("concat", p, 50)[1])
    want = reference_chunks(data, 50)
    assert got == want
    _, lines = dump("count", p)
    assert lines == [b"B %d %d" % (sum(len(s) for c in want for s in c), sum(len(c) for c in want))]


def test_invalid_utf8_lines_and_slab(tmp_path):
    rng = np.random.default_rng(2)
    data = synth_fastq(40, rng, bad_utf8_at=(3, 9))
    p = str(tmp_path / "bad.fastq")
    write(p, data, False)
    got, _, _ = parse_chunks(dump("concat", p, 7)[1])
    assert got == reference_chunks(data, 7)
    got, meta, stats = parse_chunks(dump("slab", p, 100, 512)[1])
    assert [s for c in got for s in c] == [s for c in reference_chunks(data, 100) for s in c]
    assert stats[2] == 2


def test_too_many_errors(tmp_path):
    rng = np.random.default_rng(3)
    data = synth_fastq(30, rng, bad_utf8_at=tuple(range(11)))
    p = str(tmp_path / "worse.fastq")
    write(p, data, False)
    rc, lines = dump("concat", p, 5, ok=False)
    assert rc == 3 and b"Too many read errors" in lines[-1]


def test_pos_tags_and_padding(tmp_path):
    rng = np.random.default_rng(4)
    data = synth_fastq(20, rng)
    p = str(tmp_path / "t.fastq.gz")
    write(p, data, True)
    got, meta, _ = parse_chunks(dump("slab", p, 100, 304)[1])  # the driver checks the zeroed padding
    assert [m[1] for m in meta] == [i * 7 for i in range(20)]
    assert got == reference_chunks(data, 100)


def test_error_paths(tmp_path):
    p = str(tmp_path / "long.fastq")
    write(p, b"@a\n" + b"A" * 100 + b"\n+\n" + b"I" * 100 + b"\n", False)
    rc, lines = dump("slab", p, 10, 64, ok=False)
    assert rc == 3 and lines[-1].startswith(b"ERR -2")
    rc, lines = dump("count", "/nonexistent/x.fastq.gz", ok=False)
    assert rc == 3 and b"Failed to open" in lines[-1]
    e = str(tmp_path / "e.fastq")
    write(e, b"", False)
    assert parse_chunks(dump("concat", e, 10)[1])[0] == []
    assert dump("count", e)[1] == [b"B 0 0"]


@pytest.mark.parametrize("no_libdeflate", [False, True])
def test_bgzf_lane_file(tmp_path, no_libdeflate):
    from mini_parallel_amd.synthetic import bgzf_compress
    rng = np.random.default_rng(9)
    data = synth_fastq(3000, rng, crlf=no_libdeflate)
    p = str(tmp_path / "b.fastq.gz")
    open(p, "wb").write(bgzf_compress(data))
    assert gzip.decompress(open(p, "rb").read()) == data
    env = {"MSW_NO_LIBDEFLATE": "1"} if no_libdeflate else None
    got, _, _ = parse_chunks(dump("concat", p, 333, env=env)[1])
    assert got == reference_chunks(data, 333)
    _, meta, _ = parse_chunks(dump("slab", p, 5000, 304, env=env)[1])
    assert [m[1] for m in meta] == [i * 7 for i in range(3000)]


def test_bgzf_corrupt_block(tmp_path):
    from mini_parallel_amd.synthetic import bgzf_compress
    rng = np.random.default_rng(10)
    blob = bytearray(bgzf_compress(synth_fastq(2000, rng)))
    blob[70000] ^= 0xFF
    p = str(tmp_path / "c.fastq.gz")
    open(p, "wb").write(bytes(blob))
    rc, lines = dump("concat", p, 100000, ok=False)
    assert rc == 3 and lines[-1].startswith(b"ERR")


@pytest.mark.parametrize("cap", [1, 64, 700, 1 << 20])
def test_packed_reader_any_length(tmp_path, cap):
    rng = np.random.default_rng(11)
    seqs = [bytes(rng.choice(np.frombuffer(b"ACGT", np.uint8), int(k))) for k in rng.integers(0, 5000, 60)]
    data = b"".join(b"@r%d\n%s\n+\n%s\n" % (i, s, b"I" * len(s)) for i, s in enumerate(seqs))
    p = str(tmp_path / "long.fastq.gz")
    write(p, data, True)
    _, lines = dump("packed", p, 7, cap)
    got, _, _ = parse_chunks(lines)
    assert [s.encode() for c in got for s in c] == seqs
    got, _, _ = parse_chunks(dump("concat", p, 25)[1])
    assert got == reference_chunks(data, 25)


def test_cli_flags_and_errors(tmp_path):
    """tests/test_cli.py's CPU cases (main.rs:11-46, :160-163) on the instrumented CLI."""
    r = run(CLI, ["--help"], cwd=tmp_path)
    assert r.returncode == 0
    for flag in ["--seq1", "--seq2", "--files", "--chunk-size", "--gpu", "--num-files", "--test-wgs", "--full-wgs"]:
        assert flag.encode() in r.stdout
    r = run(CLI, ["-1", "ACGT", "-2", "ACGT"], cwd=tmp_path)
    assert r.returncode == 1 and b"gpu acceleration is required" in r.stderr
    r = run(CLI, ["--full-wgs"], cwd=tmp_path)
    assert r.returncode == 1 and b"gpu acceleration is required for full WGS" in r.stderr
    r = run(CLI, ["--bogus"], cwd=tmp_path)
    assert r.returncode != 0
    r = run(CLI, ["-1", "ACGT", "-2", "ACGT", "--gpu"], cwd=tmp_path)
    assert r.returncode == 1 and b"no compatible gpu" in r.stderr
    r = run(CLI, ["--full-wgs", "--gpu"], env={"WGS_FILE_SHARD": "3/2"}, cwd=tmp_path)
    assert r.returncode == 1


def test_cli_test_wgs_and_dotenv(tmp_path):
    """--test-wgs counts bases of the lane files through the reader (main.rs:166-180,
    aligner.rs:535-544); WGS_* come from a .env file in the working directory."""
    rng = np.random.default_rng(12)
    data = synth_fastq(100, rng)
    for rr in ("R1", "R2"):
        write(str(tmp_path / f"S1_L001_{rr}_001.fastq.gz"), data, True, 2)
    (tmp_path / ".env").write_text(f"WGS_DATA_DIR={tmp_path}\nWGS_SAMPLE_ID=S1\nGPU_CHUNK_SIZE_READS=1000\n")
    r = run(CLI, ["--test-wgs"], cwd=tmp_path)
    want = sum(len(s) for c in reference_chunks(data, 1000) for s in c)
    assert r.returncode == 0
    assert r.stdout.count(b"Successfully counted %d bases" % want) == 2, r.stdout
    (tmp_path / "S1_L001_R2_001.fastq.gz").unlink()
    r = run(CLI, ["--test-wgs"], cwd=tmp_path)
    assert r.returncode == 0 and b"Error counting bases" in r.stdout


@pytest.mark.gpu
@pytest.mark.parametrize("gpu_inflate", ["0", "1"])
def test_cli_full_wgs_under_asan_on_gpu(tmp_path, oracle, gpu_inflate):
    """The instrumented host code driving the GPU (kernels uninstrumented):
    --full-wgs over BGZF lane files with two workers on the one GPU
    (MSW_DEVICES=0,0), the host reader or the GPU lane reader, async chunks,
    checkpoint and per-read records -- same per-file sums as the oracle, no
    sanitizer report.  Leak checking is off here (the HIP runtime's own
    allocations outlive main)."""
    from mini_parallel_amd.synthetic import write_wgs_dataset
    ds = write_wgs_dataset(str(tmp_path / "wgs"), lanes=2, reads_per_lane=2, reads_per_file=1500, bgzf=True)
    env = {"WGS_DATA_DIR": str(tmp_path / "wgs"), "WGS_SAMPLE_ID": "SYN", "WGS_LANES": "2",
           "WGS_READS_PER_LANE": "2", "GPU_CHUNK_SIZE_READS": "700", "WGS_RUN_ID": "asan",
           "MSW_GPU_INFLATE": gpu_inflate, "MSW_GFASTQ_BATCH": "500", "MSW_GFASTQ_SPAN_MB": "1",
           "MSW_DEVICES": "0,0",
           # no quarantine: the sanitizer runtime tracks HSA allocations too and
           # must not recycle one after the HIP runtime has unloaded at exit
           "ASAN_OPTIONS": "halt_on_error=1:detect_leaks=0:exitcode=86:quarantine_size_mb=0"}
    (tmp_path / "scores").mkdir()
    r = run(CLI, ["--full-wgs", "--gpu", "--score-mode", "sw", "--reference", ds["reference"], "--window", "300",
                  "--num-gpus", "2", "--checkpoint-dir", tmp_path, "--json", tmp_path / "rec.json",
                  "--scores-out", tmp_path / "scores"], env=env, cwd=tmp_path)
    assert r.returncode == 0, (r.stdout + r.stderr)[-3000:]
    want = 0
    for b in ds["batches"]:
        s, _, _ = oracle.sw_batch(b.reads, b.read_len, b.wins, b.win_len, threads=8)
        want += int(s.astype(np.int64).sum())
    import json
    rec = json.load(open(tmp_path / "rec.json"))
    assert rec["total_score"] == want and rec["total_reads"] == 6000
