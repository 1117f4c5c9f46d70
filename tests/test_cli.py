"""rustseq_mini (C++ CLI over the C ABI): flag surface of main.rs:11-46 and the
pair / --files / --test-wgs / --full-wgs modes against the oracle."""
import json
import os
import re
import subprocess

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CLI = os.path.join(ROOT, "mini_parallel_amd", "rustseq_mini")


def run(args, env=None, cwd=None, timeout=600):
    e = dict(os.environ)
    e.update(env or {})
    return subprocess.run([CLI] + args, capture_output=True, text=True, env=e, cwd=cwd, timeout=timeout)


def test_cli_built():
    assert os.access(CLI, os.X_OK), "rustseq_mini not built (__graft_entry__.build())"


def test_help_lists_reference_flags():
    out = run(["--help"]).stdout
    for flag in ["--seq1", "--seq2", "--files", "--chunk-size", "--gpu", "--num-files", "--test-wgs", "--full-wgs"]:
        assert flag in out


def test_requires_gpu_flag(tmp_path):
    # main.rs:160-163: no --gpu -> error + exit 1 (no CPU path)
    r = run(["-1", "ACGT", "-2", "ACGT"], cwd=tmp_path)
    assert r.returncode == 1
    assert "gpu acceleration is required" in r.stderr


def test_full_wgs_requires_gpu_flag(tmp_path):
    r = run(["--full-wgs"], cwd=tmp_path)
    assert r.returncode == 1 and "required for full WGS" in r.stderr


def test_unknown_flag(tmp_path):
    r = run(["--bogus"], cwd=tmp_path)
    assert r.returncode == 1 and "unexpected argument" in r.stderr


@pytest.mark.skipif(os.path.exists("/dev/kfd"), reason="GPU present")
def test_no_gpu_with_flag(tmp_path):
    r = run(["-1", "ACGT", "-2", "ACGT", "--gpu"], cwd=tmp_path)
    assert r.returncode == 1 and "no compatible gpu" in r.stderr


# ---------------------------------------------------------------------------
# GPU
# ---------------------------------------------------------------------------
@pytest.mark.gpu
def test_pair_compat(tmp_path):
    r = run(["-1", "ACGTACGT", "-2", "ACGTACGT", "--gpu"], cwd=tmp_path)
    assert r.returncode == 0, r.stderr
    assert "GPU Alignment score: 2" in r.stdout
    r = run(["--seq1", "AAAA", "--seq2", "CCCC", "-g"], cwd=tmp_path)
    assert "GPU Alignment score: 0" in r.stdout


@pytest.mark.gpu
def test_pair_sw(tmp_path):
    r = run(["-1", "ACGTACGT", "-2", "ACGACGT", "--gpu", "--score-mode", "sw"], cwd=tmp_path)
    assert r.returncode == 0, r.stderr
    assert "GPU Alignment score: 12" in r.stdout and "read 7, window 6" in r.stdout


def _fastq(path, seqs):
    with open(path, "w") as f:
        for i, s in enumerate(seqs):
            f.write(f"@r{i}\n{s}\n+\n{'I' * len(s)}\n")


@pytest.mark.gpu
def test_files_mode_compat(tmp_path, oracle):
    rng = np.random.default_rng(5)
    alpha = np.frombuffer(b"ACGT", np.uint8)
    s1 = [bytes(rng.choice(alpha, 150)).decode() for _ in range(25)]
    s2 = [bytes(rng.choice(alpha, 150)).decode() for _ in range(17)]
    s2[3] = s1[0]
    _fastq(tmp_path / "a.fastq", s1)
    _fastq(tmp_path / "b.fastq", s2)
    r = run(["-f", "-1", "a.fastq", "-2", "b.fastq", "--gpu"], env={"GPU_CHUNK_SIZE_READS": "10"}, cwd=tmp_path)
    assert r.returncode == 0, r.stderr
    want = 0
    c1 = ["".join(s1[i:i + 10]) for i in range(0, len(s1), 10)]
    c2 = ["".join(s2[i:i + 10]) for i in range(0, len(s2), 10)]
    for a in c1:
        for b in c2:
            want += oracle.compat_align(a.encode(), b.encode(), 1024)
    assert f"Score: {want}" in r.stdout
    assert f"Loaded {150 * 25} bases from a.fastq" in r.stdout


@pytest.mark.gpu
@pytest.mark.parametrize("bgzf,gpu_inflate", [(False, "1"), (True, "0"), (True, "1")])
def test_full_wgs_sw_and_resume(tmp_path, oracle, bgzf, gpu_inflate):
    """--full-wgs --score-mode sw over gzip or BGZF lane files (BGZF: inflated
    and parsed on the GPU -- msw_gfastq -- or, with MSW_GPU_INFLATE=0, by
    libdeflate on several host threads per file; gzip always on the host):
    per-file i64 sums and per-read records equal the oracle's,
    checkpoint/resume skips finished files."""
    from mini_parallel_amd.synthetic import write_wgs_dataset
    ds = write_wgs_dataset(str(tmp_path / "wgs"), lanes=2, reads_per_lane=2, reads_per_file=1500, bgzf=bgzf)
    env = {"WGS_DATA_DIR": str(tmp_path / "wgs"), "WGS_SAMPLE_ID": "SYN", "WGS_LANES": "2",
           "WGS_READS_PER_LANE": "2", "GPU_CHUNK_SIZE_READS": "700", "WGS_RUN_ID": "t1",
           "MSW_GPU_INFLATE": gpu_inflate, "MSW_GFASTQ_BATCH": "500", "MSW_GFASTQ_SPAN_MB": "1"}
    (tmp_path / "scores").mkdir()
    args = ["--full-wgs", "--gpu", "--score-mode", "sw", "--reference", ds["reference"], "--window", "300",
            "--checkpoint-dir", str(tmp_path), "--json", str(tmp_path / "rec.json"),
            "--scores-out", str(tmp_path / "scores")]
    r = run(args, env=env, cwd=tmp_path)
    assert r.returncode == 0, r.stdout + r.stderr
    want = 0
    per_file = []
    rec_t = np.dtype([("score", "<i4"), ("end_i", "<i2"), ("end_j", "<i2")])
    for f, b in zip(ds["files"], ds["batches"]):
        s, i, j = oracle.sw_batch(b.reads, b.read_len, b.wins, b.win_len, threads=8)
        per_file.append(int(s.astype(np.int64).sum()))
        want += per_file[-1]
        # per-read results, in file order (chunks land at their own offsets)
        got = np.fromfile(tmp_path / "scores" / (os.path.basename(f) + ".scores"), dtype=rec_t)
        assert np.array_equal(got["score"], s) and np.array_equal(got["end_i"], i) and np.array_equal(got["end_j"], j)
    rec = json.load(open(tmp_path / "rec.json"))
    assert rec["total_score"] == want and rec["total_reads"] == 6000
    # the reference's BenchmarkResult fields (tools/benchmark.rs:17-34) + GCUPS
    for k in ("timestamp", "run_id", "mode", "files_processed", "total_reads", "total_bases", "total_score",
              "total_time_seconds", "throughput_reads_per_second", "throughput_bases_per_second", "chunk_size",
              "cpu_cores_used", "parallel_files", "system_info", "gcups", "num_gpus", "host_cores"):
        assert k in rec, k
    assert rec["files_processed"] == 4 and rec["chunk_size"] == 700 and rec["gcups"] > 0
    assert rec["gpu_inflate"] == (bgzf and gpu_inflate == "1")
    assert set(rec["system_info"]) == {"gpu_name", "gpu_memory_gb", "cpu_cores", "total_ram_gb"}
    ck = json.load(open(tmp_path / "checkpoint_t1.json"))
    assert ck["completed_files"] == 4
    assert [f["score"] for f in sorted(ck["files"], key=lambda f: f["file_index"])] == per_file
    # resume: every file is skipped, totals unchanged
    r2 = run(args, env=env, cwd=tmp_path)
    assert r2.returncode == 0 and r2.stdout.count("Skipping completed file") == 4
    assert json.load(open(tmp_path / "rec.json"))["total_score"] == want


@pytest.mark.gpu
@pytest.mark.parametrize("bgzf", [False, True])
def test_full_wgs_sw_long_reads(tmp_path, oracle, bgzf):
    """--full-wgs --score-mode sw with 300 bp reads (MSW_MAX_READ_LEN=300:
    320-byte slabs; gzip lane files on the host reader, BGZF ones on the GPU
    lane reader) scored on the long-pair kernel against 600-base windows:
    per-read records and per-file sums equal the oracle's."""
    from mini_parallel_amd.synthetic import write_wgs_dataset
    ds = write_wgs_dataset(str(tmp_path / "wgs"), lanes=1, reads_per_lane=2, reads_per_file=700, read_len=300,
                           bgzf=bgzf)
    env = {"WGS_DATA_DIR": str(tmp_path / "wgs"), "WGS_SAMPLE_ID": "SYN", "WGS_LANES": "1",
           "WGS_READS_PER_LANE": "2", "GPU_CHUNK_SIZE_READS": "300", "WGS_RUN_ID": "long",
           "MSW_MAX_READ_LEN": "300"}
    (tmp_path / "scores").mkdir()
    r = run(["--full-wgs", "--gpu", "--score-mode", "sw", "--reference", ds["reference"], "--window", "600",
             "--checkpoint-dir", str(tmp_path), "--json", str(tmp_path / "rec.json"),
             "--scores-out", str(tmp_path / "scores")], env=env, cwd=tmp_path)
    assert r.returncode == 0, r.stdout + r.stderr
    want = 0
    for f, b in zip(ds["files"], ds["batches"]):
        assert int(b.read_len.max()) > 256
        s, i, j = oracle.sw_batch(b.reads, b.read_len, b.wins, b.win_len, threads=8)
        want += int(s.astype(np.int64).sum())
        got = np.fromfile(tmp_path / "scores" / (os.path.basename(f) + ".scores"), dtype=REC_T)
        assert np.array_equal(got["score"], s) and np.array_equal(got["end_i"], i) and np.array_equal(got["end_j"], j)
    rec = json.load(open(tmp_path / "rec.json"))
    assert rec["total_score"] == want and rec["total_reads"] == 1400 and rec["gpu_inflate"] == bgzf


@pytest.mark.gpu
def test_full_wgs_compat_and_test_wgs(tmp_path):
    from mini_parallel_amd.synthetic import write_wgs_dataset
    ds = write_wgs_dataset(str(tmp_path / "wgs"), lanes=1, reads_per_lane=2, reads_per_file=95)
    env = {"WGS_DATA_DIR": str(tmp_path / "wgs"), "WGS_SAMPLE_ID": "SYN", "WGS_LANES": "1",
           "WGS_READS_PER_LANE": "2", "GPU_CHUNK_SIZE_READS": "10", "WGS_RUN_ID": "t2"}
    r = run(["--full-wgs", "--gpu", "--checkpoint-dir", str(tmp_path), "--json", str(tmp_path / "c.json")],
            env=env, cwd=tmp_path)
    assert r.returncode == 0, r.stdout + r.stderr
    # each chunk self-aligned: 2 when it has >= 1000 bases (aligner.rs:365-373)
    want = 0
    for b in ds["batches"]:
        lens = b.read_len.astype(int)
        for k in range(0, len(lens), 10):
            want += 2 if lens[k:k + 10].sum() >= 1000 else 0
    assert json.load(open(tmp_path / "c.json"))["total_score"] == want
    r = run(["--test-wgs"], env=env, cwd=tmp_path)
    assert r.returncode == 0
    got = [int(x) for x in re.findall(r"Successfully counted (\d+) bases", r.stdout)]
    assert got == [int(b.read_len.astype(int).sum()) for b in ds["batches"][:2]]


REC_T = np.dtype([("score", "<i4"), ("end_i", "<i2"), ("end_j", "<i2")])


@pytest.mark.gpu
@pytest.mark.parametrize("gpu_inflate", ["0", "1"])
def test_full_wgs_config4_shape_two_workers(tmp_path, oracle, gpu_inflate):
    """BASELINE config 4's shape (8 lanes x R1/R2 lane files of 150 bp reads,
    300 bp windows), reduced to 2,000 reads per file, through the multi-worker
    path: MSW_DEVICES=0,0 --num-gpus 2 builds two contexts on the one GPU, so
    the shared chunk queue, the exactly-once file completion and per-chunk
    pwrite from several workers all run.  Per-read records and per-file i64
    sums equal the oracle's; the run record carries kernel and end-to-end
    GCUPS, HBM GB/s and both roofline fractions; resume skips every file."""
    from mini_parallel_amd.synthetic import write_wgs_dataset
    ds = write_wgs_dataset(str(tmp_path / "wgs"), lanes=8, reads_per_lane=2, reads_per_file=2000, bgzf=True,
                           workers=4)
    env = {"WGS_DATA_DIR": str(tmp_path / "wgs"), "WGS_SAMPLE_ID": "SYN", "WGS_LANES": "8",
           "WGS_READS_PER_LANE": "2", "GPU_CHUNK_SIZE_READS": "600", "WGS_RUN_ID": "c4", "MSW_DEVICES": "0,0",
           "MSW_GPU_INFLATE": gpu_inflate}
    (tmp_path / "scores").mkdir()
    args = ["--full-wgs", "--gpu", "--score-mode", "sw", "--reference", ds["reference"], "--window", "300",
            "--num-gpus", "2", "--checkpoint-dir", str(tmp_path), "--json", str(tmp_path / "rec.json"),
            "--scores-out", str(tmp_path / "scores")]
    r = run(args, env=env, cwd=tmp_path)
    assert r.returncode == 0, r.stdout + r.stderr
    per_file = []
    for f, b in zip(ds["files"], ds["batches"]):
        s, i, j = oracle.sw_batch(b.reads, b.read_len, b.wins, b.win_len, threads=16)
        per_file.append(int(s.astype(np.int64).sum()))
        got = np.fromfile(tmp_path / "scores" / (os.path.basename(f) + ".scores"), dtype=REC_T)
        assert np.array_equal(got["score"], s) and np.array_equal(got["end_i"], i) and np.array_equal(got["end_j"], j)
    rec = json.load(open(tmp_path / "rec.json"))
    assert rec["total_score"] == sum(per_file) and rec["total_reads"] == 16 * 2000
    assert rec["num_gpus"] == 2 and rec["files_processed"] == 16
    assert rec["gpu_inflate"] == (gpu_inflate == "1")
    for k in ("gcups", "gcups_end_to_end", "hbm_gbps", "roofline_fraction_hbm", "roofline_fraction_valu",
              "kernel_ms", "gpu_busy_fraction", "host_cpus_usable", "host_threads"):
        assert k in rec, k
    assert rec["gcups"] >= rec["gcups_end_to_end"] > 0
    assert 0 < rec["roofline_fraction_hbm"] < 1 and 0 < rec["roofline_fraction_valu"] < 1
    # both workers share GPU 0: their kernel time adds up on one device
    assert rec["physical_gpus"] == 1 and 0 < rec["gpu_busy_fraction"] <= 1
    assert rec["hbm_gbps"] > 0 and rec["cells"] == sum(int((b.read_len.astype(np.int64) * 300).sum())
                                                       for b in ds["batches"])
    ck = json.load(open(tmp_path / "checkpoint_c4.json"))
    assert [f["score"] for f in sorted(ck["files"], key=lambda f: f["file_index"])] == per_file
    r2 = run(args, env=env, cwd=tmp_path)
    assert r2.returncode == 0 and r2.stdout.count("Skipping completed file") == 16
    assert json.load(open(tmp_path / "rec.json"))["total_score"] == sum(per_file)


@pytest.mark.gpu
def test_full_wgs_three_files_two_workers(tmp_path, oracle):
    """three lane files on two GPU-reader workers.  A worker claims
    its next file (and pins its first window) when it opens one; a worker
    left with nothing to claim takes another worker's claimed-but-unstarted
    file.  Every file is scored exactly once, with the oracle's sums."""
    from mini_parallel_amd.synthetic import write_wgs_dataset
    ds = write_wgs_dataset(str(tmp_path / "wgs"), lanes=3, reads_per_lane=1, reads_per_file=3000, bgzf=True,
                           workers=3)
    env = {"WGS_DATA_DIR": str(tmp_path / "wgs"), "WGS_SAMPLE_ID": "SYN", "WGS_LANES": "3",
           "WGS_READS_PER_LANE": "1", "GPU_CHUNK_SIZE_READS": "1000", "WGS_RUN_ID": "three", "MSW_DEVICES": "0,0",
           "MSW_GPU_INFLATE": "1"}
    args = ["--full-wgs", "--gpu", "--score-mode", "sw", "--reference", ds["reference"], "--window", "300",
            "--num-gpus", "2", "--checkpoint-dir", str(tmp_path), "--json", str(tmp_path / "rec.json")]
    r = run(args, env=env, cwd=tmp_path)
    assert r.returncode == 0, r.stdout + r.stderr
    per_file = [int(oracle.sw_batch(b.reads, b.read_len, b.wins, b.win_len, threads=16)[0].astype(np.int64).sum())
                for b in ds["batches"]]
    rec = json.load(open(tmp_path / "rec.json"))
    assert rec["files_processed"] == 3 and rec["total_reads"] == 3 * 3000 and rec["total_score"] == sum(per_file)
    assert r.stdout.count("Processing file") == 3
    ck = json.load(open(tmp_path / "checkpoint_three.json"))
    assert [f["score"] for f in sorted(ck["files"], key=lambda f: f["file_index"])] == per_file


@pytest.mark.gpu
def test_full_wgs_file_shards(tmp_path, oracle):
    """WGS_FILE_SHARD=r/N (bench.py's config-4 leg: one process per GPU, rank
    r takes lane files r, r + N, ...): the two shards of a 2-way split cover
    every file exactly once and their per-file sums are the oracle's; the
    run record says cpu_cores_used = the CPUs the process may use
    (num_cpus::get(), tools/benchmark.rs:119); a malformed shard is refused."""
    from mini_parallel_amd.synthetic import write_wgs_dataset
    ds = write_wgs_dataset(str(tmp_path / "wgs"), lanes=3, reads_per_lane=2, reads_per_file=700, bgzf=True)
    want = {os.path.basename(f): int(oracle.sw_batch(b.reads, b.read_len, b.wins, b.win_len, threads=8)[0]
                                      .astype(np.int64).sum()) for f, b in zip(ds["files"], ds["batches"])}
    got = {}
    for r in range(2):
        env = {"WGS_DATA_DIR": str(tmp_path / "wgs"), "WGS_SAMPLE_ID": "SYN", "WGS_LANES": "3",
               "WGS_READS_PER_LANE": "2", "GPU_CHUNK_SIZE_READS": "300", "WGS_FILE_SHARD": f"{r}/2"}
        res = run(["--full-wgs", "--gpu", "--score-mode", "sw", "--reference", ds["reference"], "--window", "300",
                   "--checkpoint-dir", str(tmp_path), "--json", str(tmp_path / f"rec{r}.json")], env=env, cwd=tmp_path)
        assert res.returncode == 0, res.stdout + res.stderr
        assert f"File shard {r}/2: 3 lane file(s)" in res.stdout
        rec = json.load(open(tmp_path / f"rec{r}.json"))
        assert rec["cpu_cores_used"] == rec["host_cpus_usable"] >= 1
        ck = json.load(open(tmp_path / f"checkpoint_{rec['run_id']}.json"))
        names = [os.path.basename(x) for x in ds["files"]]
        for f in ck["files"]:
            name = os.path.basename(f["file_path"])
            assert name not in got
            got[name] = f["score"]
            # messages and the checkpoint keep the file's place in the whole lane set
            assert f["file_index"] == names.index(name) and f["file_index"] % 2 == r
            assert f"Processing file {f['file_index'] + 1}/6: " in res.stdout
            assert f"File {f['file_index'] + 1} done: " in res.stdout
    assert got == want
    env["WGS_FILE_SHARD"] = "2/2"
    res = run(["--full-wgs", "--gpu", "--score-mode", "sw", "--reference", ds["reference"]], env=env, cwd=tmp_path)
    assert res.returncode == 1 and "WGS_FILE_SHARD must be r/N" in res.stderr


@pytest.mark.gpu
def test_full_wgs_reference_formats(tmp_path, oracle):
    """The reference FASTA (read on its own thread beside the HIP init): CRLF
    line ends, a second header line splitting the sequence, blank lines and
    ragged line widths give the same bases, so the same per-file sums as the
    oracle's; a missing reference is refused with exit 1."""
    from mini_parallel_amd.synthetic import write_wgs_dataset
    ds = write_wgs_dataset(str(tmp_path / "wgs"), lanes=1, reads_per_lane=2, reads_per_file=600, bgzf=True)
    want = sum(int(oracle.sw_batch(b.reads, b.read_len, b.wins, b.win_len, threads=8)[0].astype(np.int64).sum())
               for b in ds["batches"])
    seq = "".join(l.strip() for l in open(ds["reference"]) if not l.startswith(">"))
    cut = len(seq) // 3
    odd = tmp_path / "odd.fa"
    with open(odd, "wb") as f:
        f.write(b">part one\r\n")
        for k in range(0, cut, 61):
            f.write(seq[k:min(k + 61, cut)].encode() + b"\r\n")
        f.write(b"\r\n>part two\n\n")
        rest = seq[cut:]
        f.write("\n".join(rest[k:k + 97] for k in range(0, len(rest), 97)).encode())  # no final newline
    env = {"WGS_DATA_DIR": str(tmp_path / "wgs"), "WGS_SAMPLE_ID": "SYN", "WGS_LANES": "1",
           "WGS_READS_PER_LANE": "2", "GPU_CHUNK_SIZE_READS": "300"}
    for k, ref in enumerate([ds["reference"], str(odd)]):
        r = run(["--full-wgs", "--gpu", "--score-mode", "sw", "--reference", ref, "--window", "300",
                 "--checkpoint-dir", str(tmp_path), "--json", str(tmp_path / f"rec{k}.json")],
                env=dict(env, WGS_RUN_ID=f"ref{k}"), cwd=tmp_path)
        assert r.returncode == 0, r.stdout + r.stderr
        assert f"Loaded reference: {len(seq)} bases" in r.stdout
        rec = json.load(open(tmp_path / f"rec{k}.json"))
        assert rec["total_score"] == want and rec["setup_phases"]["reference_load_ms"] > 0
    r = run(["--full-wgs", "--gpu", "--score-mode", "sw", "--reference", str(tmp_path / "missing.fa")],
            env=env, cwd=tmp_path)
    assert r.returncode == 1 and "cannot open reference" in r.stderr


@pytest.mark.gpu
def test_num_gpus_beyond_visible_fails(tmp_path):
    from mini_parallel_amd.synthetic import write_wgs_dataset
    import torch
    write_wgs_dataset(str(tmp_path / "wgs"), lanes=1, reads_per_lane=1, reads_per_file=10)
    env = {"WGS_DATA_DIR": str(tmp_path / "wgs"), "WGS_SAMPLE_ID": "SYN", "WGS_LANES": "1",
           "WGS_READS_PER_LANE": "1", "GPU_CHUNK_SIZE_READS": "10"}
    r = run(["--full-wgs", "--gpu", "--num-gpus", str(torch.cuda.device_count() + 1)], env=env, cwd=tmp_path)
    assert r.returncode == 1 and "GPU context(s) available" in r.stderr


@pytest.mark.gpu
def test_full_wgs_compat_long_reads(tmp_path):
    """Compat mode concatenates reads of any length (aligner.rs:269-276):
    MiSeq-like 2 x 300 bp reads -- and one 5 kb read -- no longer fail the
    file (the sw slabs' 256 bp stride does not apply)."""
    rng = np.random.default_rng(8)
    alpha = np.frombuffer(b"ACGT", np.uint8)
    wgs = tmp_path / "wgs"
    wgs.mkdir()
    lens = [300] * 23 + [5000] + [300] * 6
    seqs = [bytes(rng.choice(alpha, k)).decode() for k in lens]
    import gzip
    with gzip.open(wgs / "SYN_L001_R1_001.fastq.gz", "wt") as f:
        for i, s in enumerate(seqs):
            f.write(f"@r{i}\n{s}\n+\n{'I' * len(s)}\n")
    env = {"WGS_DATA_DIR": str(wgs), "WGS_SAMPLE_ID": "SYN", "WGS_LANES": "1", "WGS_READS_PER_LANE": "1",
           "GPU_CHUNK_SIZE_READS": "3", "WGS_RUN_ID": "long"}
    r = run(["--full-wgs", "--gpu", "--checkpoint-dir", str(tmp_path), "--json", str(tmp_path / "c.json")],
            env=env, cwd=tmp_path)
    assert r.returncode == 0, r.stdout + r.stderr
    rec = json.load(open(tmp_path / "c.json"))
    # every 3-read chunk has >= 1000 bases... except none: 3 x 300 = 900 < 1000, so only the chunk with the 5 kb read
    want = sum(2 for k in range(0, len(lens), 3) if sum(lens[k:k + 3]) >= 1000)
    assert rec["total_score"] == want and rec["total_reads"] == len(seqs)
    assert rec["total_bases"] == sum(lens)


@pytest.mark.gpu
def test_pair_sw_oversize_is_range_error(tmp_path):
    """A 70,000-base sequence must not wrap through the u16 length;
    past 32767 bases it is a range error."""
    r = run(["-1", "A" * 70000, "-2", "ACGT", "--gpu", "--score-mode", "sw"], cwd=tmp_path)
    assert r.returncode == 1 and "exceeds the kernel limits" in r.stderr
    r = run(["-1", "A" * 32768, "-2", "ACGT", "--gpu", "--score-mode", "sw"], cwd=tmp_path)
    assert r.returncode == 1 and "exceeds the kernel limits" in r.stderr


@pytest.mark.gpu
def test_pair_sw_long_sequences(tmp_path, oracle):
    """Pair mode with reads past the packed kernels (300 bp read, 5 kb window):
    the long-pair kernel, checked against the oracle (score and best cell)."""
    rng = np.random.default_rng(21)
    alpha = np.frombuffer(b"ACGT", np.uint8)
    w = rng.choice(alpha, 5000)
    r = w[1200:1500].copy()
    r[::37] = ord("A")
    s1, s2 = bytes(r).decode(), bytes(w).decode()
    res = run(["-1", s1, "-2", s2, "--gpu", "--score-mode", "sw"], cwd=tmp_path)
    assert res.returncode == 0, res.stdout + res.stderr
    ws, wi, wj = oracle.sw_batch(r[None, :], np.array([300], np.uint16), w[None, :], np.array([5000], np.uint16))
    assert f"GPU Alignment score: {int(ws[0])}" in res.stdout
    assert f"Best cell: read {int(wi[0])}, window {int(wj[0])}" in res.stdout
