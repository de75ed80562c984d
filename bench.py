"""Benchmark: batched deflate level 6 (+ CRC-32) on MI355X, one rank per GPU.

Metric (BASELINE.json): "compress MB/s @ level 6 + CRC32 GB/s, batched 1 MB
buffers, 1/2/4/8 GPU".

* A step = one pass of the hot path over this rank's batch: deflate level 6 of
  B independent 1 MiB Silesia-style buffers (C4's per-GPU shard: 262144 / 8 =
  32768 buffers), inputs resident in HBM (generated on the device), outputs
  written to HBM.  `value` = total input MB (1e6 B) compressed by all ranks / max
  elapsed over ranks.
* CRC-32 leg (C2: 1 M x 4 KiB random buffers on each GPU) reported as "crc32".
* roofline: the dominant deflate kernel (k_match) and the CRC kernel, timed
  live with HIP events on their launch stream; algorithmic bytes per SURVEY
  §8(d): n + out_len per deflate buffer, n + 4 per checksum buffer.
* adler32 leg (C5 shape: 16 MiB small-vocabulary buffers, 4 GiB per launch)
  reported as "adler32" with its own roofline.
* cpu_baseline (rank 0, N=1 only): the host's system zlib (the
  upstream zlib the reference vendors; its streams are checked byte-identical to
  ours, i.e. to the reference's, on the sample first) timed from C
  (oracle/libzbase.so, no Python in the loop) on a bounded sample of >= 64
  distinct buffers of the same batch, on 1 thread and on every CPU this process
  may use (the affinity set capped at the cgroup quota); `port` gives the oracle
  port (oracle/liboracle.so) on the same sample for comparison.  The crc32 and
  adler32 legs carry their own system-zlib baselines.  `host` records nproc,
  the affinity set, the cgroup CPU quota and the CPU model.
* roofline.traffic: HBM bytes per launch from the committed rocprofv3 PMC
  passes of the same launch shape (profiles/): FETCH_SIZE + WRITE_SIZE, with
  FETCH_SIZE doubled only for the streaming checksum kernels (the gfx950
  correction of the MI355X guide is for wide coalesced streaming reads).
* After timing, every stream of the default leg is checked against the
  compiled reference (length + CRC-32 of each stream on rank 0, the per-rank
  digest elsewhere; tests/golden/make_bench_shard_golden.py), 64 streams
  byte for byte against the oracle, and every status.

Multi-GPU: `--gpus N` with N > 1 and no torch.distributed environment
re-launches this script under torch.distributed.run with N ranks (a child
process, started before anything touches the GPU); under a launcher, WORLD_SIZE
must equal --gpus.  Buffers are sharded by global index (rank r takes
[r*B, (r+1)*B)), no data-path collective; after timing, one RCCL all_reduce of
{bytes in, bytes out, errors} (sum) and one of the elapsed times (max), plus an
all_gather of the per-rank stream checksums.  `--cpu-dry-run` runs the same
launcher and reductions on gloo with the oracle standing in for the GPU legs
(tests/test_dist.py).
"""
import argparse
import concurrent.futures as cf
import json
import os
import socket
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "zlib.wasm_amd"))
sys.path.insert(0, os.path.join(ROOT, "tests"))

import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

import zgpu  # noqa: E402

METRIC = "compress MB/s @ level 6 + CRC32 GB/s, batched 1 MB buffers, 1/2/4/8 GPU"
HBM_PEAK_GBS = 8000.0        # MI355X_MICROARCH.md: 8.0 TB/s spec
KIND_DATA = {
    "silesia": "synthetic: device-generated seeded Silesia-style 64 KiB-segment mix "
               "(40% prose, 20% markup, 20% binary records, 10% random, 10% runs; zgpu_gen.h, "
               "pinned by tests/golden/bench_golden.json)",
    "enwik": "synthetic: device-generated seeded enwik-style 4 KiB segments (70% word text, 30% markup)",
    "vocab": "synthetic: device-generated seeded small-vocabulary text",
    "random": "synthetic: device-generated uniform random bytes",
    "four": "synthetic: device-generated seeded 4-letter alphabet (ACGT)",
    "runs": "synthetic: device-generated seeded byte runs",
}
KIND_CONFIG = {"silesia": "C4 per-GPU shard", "enwik": "C3-style", "vocab": "C5-style", "random": "random",
               "four": "C5-style (4-letter)", "runs": "C5-style (runs)"}
KIND_ID = {"random": 0, "silesia": 1, "enwik": 2, "vocab": 3, "four": 4, "runs": 5}


def parse(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=3)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--buffers", type=int, default=int(os.environ.get("ZB_BUFFERS", 32768)),
                    help="1 MiB buffers per GPU (C4 shard = 32768)")
    ap.add_argument("--buffer-bytes", type=int, default=1 << 20)
    ap.add_argument("--level", type=int, default=6)
    ap.add_argument("--kind", default="silesia", choices=list(KIND_ID),
                    help="device generator: silesia (C4, default), enwik (C3), vocab (C5)")
    ap.add_argument("--crc-buffers", type=int, default=1 << 20)
    ap.add_argument("--crc-bytes", type=int, default=4096)
    ap.add_argument("--adler-buffers", type=int, default=256, help="C5-shaped Adler-32 leg (0: skip)")
    ap.add_argument("--adler-bytes", type=int, default=16 << 20)
    ap.add_argument("--cpu-seconds", type=float, default=10.0, help="per CPU measurement")
    ap.add_argument("--cpu-threads", type=int, default=0,
                    help="threads of the all-core CPU run (0: every CPU in the affinity set)")
    ap.add_argument("--no-cpu", action="store_true")
    ap.add_argument("--no-inflate", action="store_true", help="skip the inflate round-trip leg")
    ap.add_argument("--verify", type=int, default=64,
                    help="outputs checked bit-exact vs the oracle (at most 64 MiB of them); also the CPU sample")
    ap.add_argument("--inflight-mb", type=int, default=4096,
                    help="input bytes per deflate sub-batch (workspace ~15 B per byte)")
    ap.add_argument("--cpu-dry-run", action="store_true",
                    help="test mode: gloo + oracle instead of the GPU legs (launcher/reduction check)")
    ap.add_argument("--plan-only", action="store_true",
                    help="print each rank's HBM / host memory plan for these arguments and exit (no compute)")
    return ap.parse_args(argv)


# ------------------------------------------------------------------ launch

def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def launch_cmd(a, argv):
    """torch.distributed.run command that runs this script on a.gpus ranks."""
    return [sys.executable, "-m", "torch.distributed.run", "--nnodes=1",
            f"--nproc-per-node={a.gpus}", "--master-addr=127.0.0.1",
            f"--master-port={_free_port()}", os.path.abspath(__file__)] + list(argv)


def maybe_launch(a, argv):
    """--gpus N > 1 without a launcher: start N ranks as a child process (no GPU
    has been touched in this process) and exit with its status."""
    if a.gpus > 1 and "WORLD_SIZE" not in os.environ:
        rc = subprocess.call(launch_cmd(a, argv))
        sys.exit(rc)


class Dist:
    """Rank layout and the end-of-run collectives.  nccl (RCCL over xGMI) on the
    GPU; gloo in --cpu-dry-run."""

    def __init__(self, a):
        self.world = int(os.environ.get("WORLD_SIZE", "1"))
        self.rank = int(os.environ.get("RANK", "0"))
        self.local = int(os.environ.get("LOCAL_RANK", "0"))
        if self.world != a.gpus:
            raise SystemExit(f"bench.py: --gpus {a.gpus} but WORLD_SIZE={self.world}")
        self.cpu = a.cpu_dry_run
        self.dev = torch.device("cpu") if self.cpu else torch.device("cuda", self.local)
        if not self.cpu:
            torch.cuda.set_device(self.local)
        self.backend = None
        # under a launcher the collectives run even with one rank, so the RCCL
        # path is the one a single-GPU box exercises too (tests/test_gpu.py)
        self.pg = self.world > 1 or "MASTER_ADDR" in os.environ
        if self.pg:
            if self.cpu:
                dist.init_process_group("gloo")
            else:
                dist.init_process_group("nccl", device_id=self.dev)
            self.backend = dist.get_backend()
            assert dist.get_world_size() == self.world

    def barrier(self):
        if self.pg:
            dist.barrier()
        if not self.cpu:
            torch.cuda.synchronize()

    def _reduce(self, vals, op):
        if not self.pg:
            return [float(v) for v in vals]
        t = torch.tensor([float(v) for v in vals], dtype=torch.float64, device=self.dev)
        dist.all_reduce(t, op=op)
        return t.tolist()

    def sum(self, *vals):
        return self._reduce(vals, dist.ReduceOp.SUM)

    def max(self, *vals):
        return self._reduce(vals, dist.ReduceOp.MAX)

    def gather(self, vals):
        """all_gather of a fixed-length int64 vector per rank."""
        t = torch.tensor(vals, dtype=torch.int64, device=self.dev)
        if not self.pg:
            return [t.tolist()]
        out = [torch.empty_like(t) for _ in range(self.world)]
        dist.all_gather(out, t)
        return [o.tolist() for o in out]

    def close(self):
        if self.pg:
            dist.destroy_process_group()


def shard(rank, world, per_gpu):
    """Global buffer indices owned by `rank`: a contiguous block of `per_gpu`
    (weak scaling: per-GPU work is fixed, the job grows with N)."""
    return rank * per_gpu, (rank + 1) * per_gpu


# ------------------------------------------------------------------ GPU legs

def deflate_leg(a, D):
    n, B = a.buffer_bytes, a.buffers
    first, _ = shard(D.rank, D.world, B)
    cap = (zgpu.compress_bound(n) + 15) // 16 * 16
    src = torch.empty(n * B, dtype=torch.uint8, device="cuda")
    zgpu.generate_dev(src, n, B, KIND_ID[a.kind], seed=2025, first_index=first)
    off = torch.arange(B, dtype=torch.int64, device="cuda") * n
    ln = torch.full((B,), n, dtype=torch.int64, device="cuda")
    dst = torch.empty(cap * B, dtype=torch.uint8, device="cuda")
    doff = torch.arange(B, dtype=torch.int64, device="cuda") * cap
    dcap = torch.full((B,), cap, dtype=torch.int64, device="cuda")
    dlen = torch.zeros(B, dtype=torch.int64, device="cuda")
    st = torch.full((B,), 99, dtype=torch.int32, device="cuda")

    def step():
        zgpu.deflate_batch_dev(src, off, ln, dst, doff, dcap, dlen, st, level=a.level)

    for _ in range(a.warmup):
        step()
    D.barrier()
    zgpu.stage_timing(True)
    t0 = time.perf_counter()
    for _ in range(a.steps):
        step()
    D.barrier()
    el = time.perf_counter() - t0
    zgpu.stage_timing(False)
    stages = zgpu.stage_timing_read()
    errors = int((st != 0).sum().item())
    out_bytes = int(dlen.sum().item())
    # per-rank digest of the output: sum of stream lengths and XOR of stream CRCs
    scrc = torch.zeros(B, dtype=torch.int32, device="cuda")
    zgpu.crc32_batch_dev(dst, doff, dlen, scrc)
    digest = _xor_all(scrc)
    return dict(src=src, dst=dst, dlen=dlen, cap=cap, elapsed=el, stages=stages, errors=errors,
                out_bytes=out_bytes, in_bytes=n * B, digest=digest, scrc=scrc, first=first)


def shard_golden_check(a, D, d):
    """Every stream of the default deflate leg against the compiled reference
    (tests/golden/make_bench_shard_golden.py): on rank 0 each stream's length
    and the CRC-32 of its bytes (computed on the device, k_crc32s) must equal
    the reference's compress2() stream's; on other ranks the per-rank digest
    (sum of lengths, XOR of CRCs).  Returns (streams checked, digest checked,
    note); only the bench's own configuration has goldens."""
    import numpy as np
    gdir = os.path.join(ROOT, "tests", "golden")
    try:
        doc = json.load(open(os.path.join(gdir, "bench_shard_golden.json")))
    except OSError:
        return 0, False, "no tests/golden/bench_shard_golden.json"
    if (a.kind, a.buffer_bytes, a.buffers, a.level) != (doc["kind"], doc["buffer_bytes"], doc["buffers_per_rank"],
                                                         doc["level"]):
        return 0, False, "no golden for this configuration (kind, buffer size, buffers, level)"
    lens = d["dlen"].cpu().numpy().astype(np.uint64)
    crcs = d["scrc"].cpu().numpy().view(np.uint32)
    checked, dig = 0, False
    r = str(D.rank)
    if r in doc["ranks"]:
        want = doc["ranks"][r]
        got = {"out_bytes": int(lens.sum()), "stream_crc_xor": "%08x" % int(np.bitwise_xor.reduce(crcs))}
        assert got == want, f"rank {r}: stream digest {got} != reference {want}"
        dig = True
    if D.rank == 0 and os.path.exists(os.path.join(gdir, "bench_shard_golden_r0.npz")):
        g = np.load(os.path.join(gdir, "bench_shard_golden_r0.npz"), allow_pickle=False)
        bad = np.nonzero((g["lens"].astype(np.uint64) != lens) | (g["crcs"] != crcs))[0]
        assert bad.size == 0, f"{bad.size} streams differ from the reference's (first: buffer {int(bad[0])})"
        checked = int(lens.size)
    return checked, dig, f"reference {doc.get('reference')}"


def _xor_all(t):
    import numpy as np
    return int(np.bitwise_xor.reduce(t.cpu().numpy().view("uint32")))


def checksum_leg(a, D, which):
    """C2 (CRC-32, 1 M x 4 KiB random) or the C5-shaped Adler-32 leg (16 MiB
    small-vocabulary buffers), timed with events on the launch stream."""
    if which == "crc32":
        n, B, kind, seed, fn = a.crc_bytes, a.crc_buffers, zgpu.KIND_RANDOM, 77, zgpu.crc32_batch_dev
    else:
        n, B, kind, seed, fn = a.adler_bytes, a.adler_buffers, zgpu.KIND_SMALLVOCAB, 91, zgpu.adler32_batch_dev
    first, _ = shard(D.rank, D.world, B)
    src = torch.empty(n * B, dtype=torch.uint8, device="cuda")
    zgpu.generate_dev(src, n, B, kind, seed=seed, first_index=first)
    off = torch.arange(B, dtype=torch.int64, device="cuda") * n
    ln = torch.full((B,), n, dtype=torch.int64, device="cuda")
    out = torch.zeros(B, dtype=torch.int32, device="cuda")
    stream = torch.cuda.current_stream()
    for _ in range(max(1, a.warmup)):
        fn(src, off, ln, out)
    D.barrier()
    evs = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
           for _ in range(a.steps)]
    t0 = time.perf_counter()
    for e0, e1 in evs:
        e0.record(stream)
        fn(src, off, ln, out)
        e1.record(stream)
    D.barrier()
    el = time.perf_counter() - t0
    kms = sum(e0.elapsed_time(e1) for e0, e1 in evs) / len(evs)
    return dict(src=src, out=out, elapsed=el, kernel_ms=kms, bytes=n * B, n=n, B=B)


def inflate_leg(a, D, d):
    """Decompress every stream the deflate leg produced (the other half of the
    wire format) and check the full-size round trip on the
    device: inflate(deflate(x)) == x for all buffers, every status Z_OK."""
    n, B = a.buffer_bytes, a.buffers
    src, dst, dlen, cap = d["src"], d["dst"], d["dlen"], d["cap"]
    soff = torch.arange(B, dtype=torch.int64, device="cuda") * cap
    out = torch.empty(n * B, dtype=torch.uint8, device="cuda")
    ooff = torch.arange(B, dtype=torch.int64, device="cuda") * n
    ocap = torch.full((B,), n, dtype=torch.int64, device="cuda")
    olen = torch.zeros(B, dtype=torch.int64, device="cuda")
    ost = torch.full((B,), 99, dtype=torch.int32, device="cuda")

    def step():
        zgpu.inflate_batch_dev(dst, soff, dlen, out, ooff, ocap, olen, ost)

    for _ in range(max(1, a.warmup)):
        step()
    out.zero_()
    D.barrier()
    zgpu.stage_timing(True)
    t0 = time.perf_counter()
    for _ in range(a.steps):
        step()
    D.barrier()
    el = time.perf_counter() - t0
    zgpu.stage_timing(False)
    stages = zgpu.stage_timing_read()
    ok = int((ost != 0).sum().item()) == 0 and bool((olen == n).all().item()) and bool(torch.equal(out, src))
    assert ok, "inflate(deflate(x)) != x on the device"
    del out
    return dict(elapsed=el, stages=stages, out_bytes=n * B, in_bytes=int(dlen.sum().item()))


def dry_deflate_leg(a, D):
    """--cpu-dry-run: the oracle compresses this rank's shard of host buffers
    made by the device generator's host twin (oracle/zgen.c: same kind, seed
    and global indices as the GPU leg), so the launcher, the sharding and the
    collectives run for real without a GPU, and the per-rank digests can be
    compared with the compiled reference's (tests/golden/bench_shard_golden_small.json)."""
    import zlib as _z
    from zhelpers import Oracle
    o = Oracle()
    first, last = shard(D.rank, D.world, a.buffers)
    t0 = time.perf_counter()
    in_b = out_b = digest = 0
    for _ in range(a.steps):
        in_b = out_b = digest = 0
        for g in range(first, last):
            data = o.generate(a.buffer_bytes, 1, KIND_ID[a.kind], 2025, g)[0]
            z = o.compress(data, a.level)[1]
            in_b += len(data)
            out_b += len(z)
            digest ^= _z.crc32(z)
    return dict(elapsed=time.perf_counter() - t0, in_bytes=in_b, out_bytes=out_b, errors=0,
                digest=digest, stages={})


def dry_digest_check(a, digests):
    """--cpu-dry-run: every rank's digest against the compiled reference's for
    the same configuration (tests/golden/make_bench_shard_golden_small.py), if
    there is one.  Returns (ranks checked, note)."""
    try:
        doc = json.load(open(os.path.join(ROOT, "tests", "golden", "bench_shard_golden_small.json")))
    except OSError:
        return 0, "no tests/golden/bench_shard_golden_small.json"
    if (a.kind, a.buffer_bytes, a.buffers, a.level) != (doc["kind"], doc["buffer_bytes"], doc["buffers_per_rank"],
                                                         doc["level"]):
        return 0, "no small golden for this configuration"
    n = 0
    for r, (dg, ob) in enumerate(digests):
        want = doc["ranks"].get(str(r))
        if want is None:
            continue
        got = {"out_bytes": int(ob), "stream_crc_xor": "%08x" % (int(dg) & 0xffffffff)}
        assert got == want, f"rank {r}: dry-run digest {got} != reference {want}"
        n += 1
    return n, f"reference {doc.get('reference')}"


# Device memory of one rank (bytes), from the library's allocations (DESIGN.md
# 3): the L4-9 pipelined deflate keeps, per in-flight input byte, link 2 + key
# 1 + rfull 4 + rquart 4 + pstate 1/4 in two slots and sym 4 + stage 4 in one
# (30.5 B), every workspace allocated with 1/8 slack (zgpu_api.cpp DevBuf);
# the inflate leg adds its output and ~2.7 B of match records per in-flight
# output byte; the checksum legs their inputs.  Workspaces are kept for the
# context's life, so the legs add up.
WS_PER_INFLIGHT_BYTE = 30.5 * 1.125
INFL_WS_PER_INFLIGHT_BYTE = 2.7 * 1.125
HBM_BYTES_MI355X = 288e9


def memory_plan(a, world):
    n, B = a.buffer_bytes, a.buffers
    cap = (n + (n >> 12) + (n >> 14) + (n >> 25) + 13 + 15) // 16 * 16       # compressBound, 16-B rounded
    inflight = min(a.inflight_mb << 20, n * B) if a.level >= 4 else min(4 * (a.inflight_mb << 20), n * B)
    ws = WS_PER_INFLIGHT_BYTE * inflight if a.level >= 4 else 6.0 * 1.125 * inflight
    legs = {
        "deflate_inputs": n * B,
        "deflate_outputs": cap * B,
        "deflate_workspace": int(ws),
        "inflate_outputs": 0 if a.no_inflate else n * B,
        "inflate_workspace": 0 if a.no_inflate else int(INFL_WS_PER_INFLIGHT_BYTE * min(a.inflight_mb << 20, n * B)),
        "crc32_inputs": a.crc_buffers * a.crc_bytes,
        "adler32_inputs": a.adler_buffers * a.adler_bytes,
    }
    need = sum(legs.values())
    have = HBM_BYTES_MI355X
    src = "MI355X nominal 288 GB"
    if not a.cpu_dry_run and not a.plan_only and torch.cuda.is_available():
        have = float(torch.cuda.mem_get_info()[1])
        src = "torch.cuda.mem_get_info"
    # host side per rank: the interpreter, torch and the library (~3 GB
    # resident), the verification sample (<= 64 MiB) and, on rank 0 of a
    # 1-GPU run, the CPU baseline's sample and outputs
    host = 3e9 + min(64 << 20, n * B) * 3
    try:
        avail = 0
        for line in open("/proc/meminfo"):
            if line.startswith("MemAvailable:"):
                avail = int(line.split()[1]) * 1024
    except OSError:
        avail = None
    return {"hbm_bytes_per_rank": {k: int(v) for k, v in legs.items()}, "hbm_need_per_rank": int(need),
            "hbm_have_per_rank": int(have), "hbm_source": src, "hbm_fits": need <= have,
            "host_bytes_per_rank_est": int(host), "host_need_all_ranks_est": int(host * world),
            "host_available": avail,
            "host_fits": None if avail is None else host * world <= avail}


# ------------------------------------------------------------------ CPU baselines

def host_info():
    info = {"nproc": os.cpu_count(), "affinity_cpus": len(os.sched_getaffinity(0))}
    try:
        info["cgroup_cpu_max"] = open("/sys/fs/cgroup/cpu.max").read().strip()
    except OSError:
        info["cgroup_cpu_max"] = None
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                info["cpu_model"] = line.split(":", 1)[1].strip()
                break
    except OSError:
        pass
    return info


def _timed_threads(fn, sample, threads, seconds):
    """Run fn(buffer) over the sample, round-robin, on `threads` threads for
    about `seconds`; returns (MB/s, bytes done).  fn releases the GIL (ctypes
    calls, zlib.compress)."""
    deadline = time.perf_counter() + seconds

    def work(tid):
        done, k = 0, tid
        while time.perf_counter() < deadline:
            b = sample[k % len(sample)]
            fn(b)
            done += len(b)
            k += threads
        return done

    t0 = time.perf_counter()
    with cf.ThreadPoolExecutor(threads) as ex:
        total = sum(ex.map(work, range(threads)))
    return total / (time.perf_counter() - t0) / 1e6, total


def progress(msg):
    """A progress line on stderr (a long CPU or verification phase stays visibly alive)."""
    print(f"[bench {time.strftime('%H:%M:%S')}] {msg}", file=sys.stderr, flush=True)


def _zbase():
    """oracle/libzbase.so: system zlib timed from C threads (bench infrastructure)."""
    import ctypes as C
    lib = C.CDLL(os.path.join(ROOT, "oracle", "libzbase.so"))
    lib.zb_compress_rate.restype = C.c_double
    lib.zb_compress_rate.argtypes = [C.POINTER(C.c_void_p), C.POINTER(C.c_size_t), C.c_int, C.c_int, C.c_int,
                                     C.c_double, C.POINTER(C.c_uint64)]
    for f in (lib.zb_crc32_rate, lib.zb_adler32_rate):
        f.restype = C.c_double
        f.argtypes = [C.c_void_p, C.c_size_t, C.c_size_t, C.c_int, C.c_double, C.POINTER(C.c_uint64)]
    lib.zb_zlib_version.restype = C.c_char_p
    return lib


def cpu_threads(a):
    """(threads, host info, quota): every CPU this process may use -- the affinity
    set, capped at the cgroup CPU quota when there is one (more threads than the
    quota's CPUs share the same CPU time and only stretch the run)."""
    host = host_info()
    quota = None
    try:
        q, per = host["cgroup_cpu_max"].split()
        quota = None if q == "max" else round(int(q) / int(per), 2)
    except (AttributeError, ValueError):
        pass
    allt = a.cpu_threads or host["affinity_cpus"]
    if not a.cpu_threads and quota:
        allt = max(1, min(allt, int(quota + 0.999)))
    return allt, host, quota


def cpu_baselines(a, sample, want, level):
    """System zlib and the oracle port on 1 thread and on all
    CPUs this process may use; SURVEY §8(d) / BASELINE.md §3."""
    import ctypes as C
    import zlib
    from zhelpers import Oracle
    o = Oracle()
    allt, host, quota = cpu_threads(a)
    secs = a.cpu_seconds
    zb = _zbase()
    ver = zb.zb_zlib_version().decode()
    bufs = [C.create_string_buffer(b, len(b)) for b in sample]
    ptrs = (C.c_void_p * len(bufs))(*[C.cast(b, C.c_void_p) for b in bufs])
    lens = (C.c_size_t * len(bufs))(*[len(b) for b in sample])
    done = C.c_uint64(0)
    ident = all(zlib.compress(b, level) == z for b, z in zip(sample, want))
    mb = sum(len(b) for b in sample) / 1e6
    progress(f"cpu baseline: system zlib {ver}, 1 thread then {allt} ({len(sample)} buffers, {mb:.0f} MB)")
    sys1 = zb.zb_compress_rate(ptrs, lens, len(bufs), level, 1, secs / 2, C.byref(done))
    sysn = zb.zb_compress_rate(ptrs, lens, len(bufs), level, allt, secs, C.byref(done))
    sysn_b = done.value
    err = None
    if sys1 < 0 or sysn < 0:     # a zlib call or an allocation failed inside zb_compress_rate
        err = f"system zlib compress2 failed in the timing loop (1 thread: {sys1}, {allt} threads: {sysn})"
    progress(f"cpu baseline: oracle port, 1 thread then {allt}")
    port1, _ = _timed_threads(lambda b: o.compress(b, level), sample, 1, secs / 4)
    portn, portn_b = _timed_threads(lambda b: o.compress(b, level), sample, allt, secs / 2)
    if err:
        return {"value": None, "unit": "MB/s", "cores": allt, "kind": "reference", "error": err,
                "port": {"value": round(portn, 2), "per_core_1thread": round(port1, 2), "cores": allt},
                "host": host}
    return {"value": round(sysn, 2), "unit": "MB/s", "cores": allt,
            "kind": "reference",
            "kind_note": f"system zlib {ver} compress2() (upstream zlib: the deflate.c/trees.c the reference "
                         f"vendors as zlib 1.3.1.1-motley; BASELINE.md §3.1), "
                         + ("byte-identical to this run's GPU streams on every sample buffer"
                            if ident else "NOT byte-identical on the sample"),
            "bit_identical_on_sample": ident,
            "cpu_quota_cpus": quota,
            "per_core_1thread": round(sys1, 2),
            "all_host_cpus_linear_estimate": round(sys1 * host["nproc"], 1),
            "sample": f"{len(sample)} distinct {a.buffer_bytes} B {a.kind} buffers of this batch "
                      f"(evenly strided indices, the ones verified bit-exact), compressed repeatedly at level "
                      f"{level} from C threads: ~{secs / 2:.0f} s on 1 thread, ~{secs:.0f} s "
                      f"({sysn_b / 1e6:.0f} MB) on {allt} threads (the CPUs this process may use: affinity "
                      f"set capped at the cgroup quota)",
            "port": {"value": round(portn, 2), "per_core_1thread": round(port1, 2), "cores": allt,
                     "note": f"oracle/liboracle.so (our C restatement of deflate.c/trees.c) on the same sample, "
                             f"{portn_b / 1e6:.0f} MB"},
            "host": host}


def checksum_cpu_baseline(a, which, c):
    """System zlib crc32()/adler32() over the leg's own buffers (the first 64 MiB
    of them, in the leg's buffer size) on 1 thread and on all CPUs this process
    may use."""
    import ctypes as C
    allt, _, _ = cpu_threads(a)
    nb = max(1, min(c["B"], (64 << 20) // c["n"]))
    host = c["src"][:nb * c["n"]].cpu().numpy()
    buf = C.create_string_buffer(host.tobytes(), nb * c["n"])
    zb = _zbase()
    fn = zb.zb_crc32_rate if which == "crc32" else zb.zb_adler32_rate
    done = C.c_uint64(0)
    secs = max(1.0, a.cpu_seconds / 4)
    one = fn(buf, nb * c["n"], c["n"], 1, secs / 2, C.byref(done))
    alln = fn(buf, nb * c["n"], c["n"], allt, secs, C.byref(done))
    if one < 0 or alln < 0:
        return {"value": None, "unit": "GB/s", "cores": allt, "kind": "reference",
                "error": f"system zlib {which}() timing failed (1 thread: {one}, {allt} threads: {alln})"}
    out = {"value": round(alln / 1e3, 3), "unit": "GB/s", "cores": allt, "kind": "reference",
           "kind_note": f"system zlib {zb.zb_zlib_version().decode()} {which}()",
           "per_core_1thread": round(one / 1e3, 3),
           "sample": f"{nb} x {c['n']} B buffers of this leg, one {which}() call per buffer, repeatedly: "
                     f"~{secs / 2:.1f} s on 1 thread, ~{secs:.1f} s ({done.value / 1e9:.1f} GB) on {allt} threads"}
    if which == "crc32":
        out["reference_braided_crc32_per_core_container"] = {
            "value": 2.26, "unit": "GB/s",
            "note": "the reference's zlib 1.3.1.1 braided crc32 measured in the build container (BASELINE.md §2); "
                    "system zlib 1.2.11's crc32 is about 2x slower"}
    return out


# ------------------------------------------------------------------ reporting

def shipped_kernels():
    """Kernel instances compiled into the current libzgpu.so ("k_match<false, false>", ...),
    from the host-side launch stubs."""
    import re
    out = subprocess.run(["nm", "-C", os.path.join(ROOT, "zlib.wasm_amd", "libzgpu.so")],
                         capture_output=True, text=True).stdout
    return set(m.group(1) for m in re.finditer(r"__device_stub__(k_[A-Za-z0-9_]+(?:<[^>]*>)?)\(", out))


def pmc_traffic(kernels, tag, streaming=False):
    """HBM bytes per launch of a leg from the committed rocprofv3 PMC passes
    (profiles/*_pmc_fetch_*.csv, *_pmc_write_*.csv, units KiB).  FETCH_SIZE is
    doubled only for `streaming` kernels: the MI355X guide's gfx950 correction
    holds for wide coalesced streaming reads (MI355X_MICROARCH.md, HBM), not for
    the random 4-byte and line-sized reads of the deflate kernels, whose raw
    FETCH_SIZE is reported (the doubled figure beside it as an upper bound).
    Returns (bytes, source, detail).  Only for profiles taken on
    this launch's shape (the file name carries the shape tag).  `kernels`: the
    name prefixes of the kernels one launch of the leg runs; for each, only the
    dispatches with its largest grid (the leg's own launches, not the small
    verification or trailer launches of the same kernel) are averaged.  A
    profile of a kernel instance the current library does not ship (a renamed
    template, an old A/B variant) is refused: the figure must be of the timed
    kernel."""
    import csv
    import glob
    fetch = sorted(glob.glob(os.path.join(ROOT, "profiles", f"*_pmc_fetch_*{tag}*.csv")))
    write = sorted(glob.glob(os.path.join(ROOT, "profiles", f"*_pmc_write_*{tag}*.csv")))
    if not fetch or not write:
        return None, None, None
    shipped = shipped_kernels()

    def name(r):
        return r["Kernel_Name"].split("(")[0].replace("void ", "").replace("zgpu::", "")

    def per_launch(path, counter):
        total = 0.0
        rows = [r for r in csv.DictReader(open(path)) if r["Counter_Name"] == counter]
        for k in kernels:
            mine = [r for r in rows if name(r).startswith(k)]
            if not mine:
                return None
            g = max(int(r["Grid_Size"]) for r in mine)
            top = [r for r in mine if int(r["Grid_Size"]) == g]
            if any(name(r) not in shipped for r in top):
                return None
            vals = [float(r["Counter_Value"]) for r in top]
            total += sum(vals) / len(vals) * 1024.0
        return total

    f = per_launch(fetch[-1], "FETCH_SIZE")
    w = per_launch(write[-1], "WRITE_SIZE")
    if f is None or w is None:
        return None, None, None
    detail = {"fetch_size_raw": int(f), "write_size": int(w), "fetch_x2_applied": bool(streaming),
              "with_fetch_x2": int(2.0 * f + w)}
    return (2.0 * f if streaming else f) + w, os.path.basename(fetch[-1]) + " + " + os.path.basename(write[-1]), detail


def launches_tag(a):
    """Shape of one deflate launch (sub-batch): buffers x bytes."""
    # levels 1-3 keep 4x the in-flight budget (zgpu_api.cpp deflate_dev_locked)
    mult = 4 if 1 <= a.level <= 3 else 1
    per = max(1, min(a.buffers, mult * (a.inflight_mb << 20) // a.buffer_bytes))
    return f"{per}x{a.buffer_bytes}"


def checksum_report(a, c, D, which, tag, cpu=None):
    el, = D.max(c["elapsed"])
    tot, = D.sum(float(c["bytes"]) * a.steps)
    alg = (c["n"] + 4) * c["B"]
    gbs = alg / (c["kernel_ms"] / 1e3) / 1e9
    kern = "k_crc32" if which == "crc32" else "k_adler32"
    # the kernels one launch runs: 16 lanes per buffer for C2's 1 M buffers;
    # pieces + combine for the C5 leg's few large buffers (zgpu_checksum.hip)
    parts = ["k_crc32s<16>"] if which == "crc32" else ["k_adler32_part", "k_adler32_fin"]
    traffic, src, tdet = pmc_traffic(parts, tag, streaming=True)
    return {"value": round(tot / el / 1e9, 2), "unit": "GB/s",
            "roofline": {"bound": "hbm", "kernel": kern, "achieved": round(gbs, 1), "peak": HBM_PEAK_GBS,
                         "unit": "GB/s", "frac": round(gbs / HBM_PEAK_GBS, 4),
                         "traffic": None if traffic is None else int(traffic), "traffic_source": src,
                         "traffic_detail": tdet,
                         "alg_bytes_per_launch": alg, "avg_launch_ms": round(c["kernel_ms"], 4)},
            "cpu_baseline": cpu}


def main(argv=None):
    argv = sys.argv[1:] if argv is None else argv
    a = parse(argv)
    if a.plan_only:
        # no launcher, no GPU: the plan of every rank of a --gpus N run
        plan = memory_plan(a, a.gpus)
        print(json.dumps({"memory_plan": plan, "n_gpus": a.gpus, "ranks_same_plan": True}), flush=True)
        return
    maybe_launch(a, argv)
    D = Dist(a)

    if a.cpu_dry_run:
        d = dry_deflate_leg(a, D)
        inf = c = ad = None
    else:
        assert zgpu.load().zgpu_init() == 0, "libzgpu: GPU init failed"
        zgpu.set_inflight_bytes(a.inflight_mb << 20)
        progress("deflate leg")
        d = deflate_leg(a, D)
        progress("inflate leg")
        inf = None if a.no_inflate else inflate_leg(a, D, d)
        progress("checksum legs")
        c = checksum_leg(a, D, "crc32")
        ad = checksum_leg(a, D, "adler32") if a.adler_buffers > 0 else None

    # ---- the end-of-run collectives (the only ones: no data-path exchange) ----
    el, = D.max(d["elapsed"])
    in_total, out_total, errors = D.sum(float(d["in_bytes"]) * a.steps, float(d["out_bytes"]),
                                        float(d["errors"]))
    digests = D.gather([int(d["digest"]), int(d["out_bytes"])])
    assert errors == 0, f"deflate status != Z_OK on {int(errors)} buffers"

    # ---- verification on this rank (outside the timed region) ----
    if a.cpu_dry_run:
        dry_ranks, dry_note = dry_digest_check(a, digests)
        shard_n, shard_dig, shard_note = 0, dry_ranks == D.world, "cpu dry run: " + dry_note
    else:
        shard_n, shard_dig, shard_note = shard_golden_check(a, D, d)
    from zhelpers import Oracle
    o = Oracle()
    sample, want = [], []
    n = a.buffer_bytes
    if not a.cpu_dry_run:
        h_dlen = d["dlen"].cpu().numpy()
        nver = min(a.verify, max(1, (64 << 20) // n))
        idx = sorted(set(int(i) for i in torch.linspace(0, a.buffers - 1, nver).tolist())) \
            if a.verify > 0 else []
        for i in idx:
            progress(f"verifying buffer {i} against the oracle")
            raw = d["src"][i * n:(i + 1) * n].cpu().numpy().tobytes()
            z = d["dst"][i * d["cap"]: i * d["cap"] + int(h_dlen[i])].cpu().numpy().tobytes()
            assert z == o.compress(raw, a.level)[1], f"buffer {i}: GPU stream != oracle"
            sample.append(raw)
            want.append(z)
        crc_h = c["out"][:64].cpu().numpy().view("uint32")
        for i in range(64):
            raw = c["src"][i * a.crc_bytes:(i + 1) * a.crc_bytes].cpu().numpy().tobytes()
            assert int(crc_h[i]) == o.crc32(raw), f"crc buffer {i} mismatch"
        if ad is not None:
            ad_h = ad["out"][:2].cpu().numpy().view("uint32")
            for i in range(min(2, ad["B"])):
                raw = ad["src"][i * ad["n"]:(i + 1) * ad["n"]].cpu().numpy().tobytes()
                assert int(ad_h[i]) == o.adler32(raw), f"adler buffer {i} mismatch"

    if inf is not None:
        inf_el, = D.max(inf["elapsed"])
        inf_total, = D.sum(float(inf["out_bytes"]) * a.steps)
    cpu_on = not a.no_cpu and not a.cpu_dry_run and D.world == 1 and D.rank == 0
    crc = None if c is None else checksum_report(a, c, D, "crc32", f"C2_{a.crc_buffers}x{a.crc_bytes}",
                                                 checksum_cpu_baseline(a, "crc32", c) if cpu_on else None)
    adl = None if ad is None else checksum_report(a, ad, D, "adler32", f"A5_{a.adler_buffers}x{a.adler_bytes}",
                                                  checksum_cpu_baseline(a, "adler32", ad) if cpu_on else None)

    if D.rank == 0:
        mbps = in_total / el / 1e6
        ratio = in_total / a.steps / max(1.0, out_total)
        st = d["stages"]
        roof = None
        # dominant kernel: k_match ("match") at L4-9, k_parse_fast ("parse_greedy")
        # at L1-3; algorithmic bytes per launch = Σ (n + out_len) over the
        # buffers one launch processes
        dom = None
        if st.get("match", (0, 0))[1] > 0:
            dom = ("match", "k_match<", "k_match",
                   "not HBM: dependent LDS round trips of the chain walks and instruction issue (DESIGN.md 4.3)")
        elif st.get("parse_greedy", (0, 0))[1] > 0:
            dom = ("parse_greedy", "k_parse_fast<", "k_parse_fast",
                   "not HBM: one wave-uniform sequential parse per buffer (deflate_fast), bound by scalar "
                   "instruction issue on the CU's one scalar unit (DESIGN.md 4.5)")
        if dom is not None:
            mms, mcount = st[dom[0]]
            per_step_alg = d["in_bytes"] + d["out_bytes"]
            launches_per_step = max(1, mcount // max(1, a.steps))
            alg_per_launch = per_step_alg / launches_per_step
            m_avg_ms = mms / max(1, mcount)
            achieved = alg_per_launch / (m_avg_ms / 1e3) / 1e9 if m_avg_ms > 0 else 0.0
            m_traffic, m_src, m_det = pmc_traffic([dom[1]], f"L{a.level}_{launches_tag(a)}")
            roof = {"bound": "hbm", "kernel": dom[2],
                    "achieved": round(achieved, 2), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                    "frac": round(achieved / HBM_PEAK_GBS, 6),
                    "traffic": None if m_traffic is None else int(m_traffic),
                    "traffic_source": m_src,
                    "traffic_detail": m_det,
                    "alg_bytes_per_launch": int(alg_per_launch),
                    "avg_launch_ms": round(m_avg_ms, 3),
                    "limiter": dom[3]}
        cpu = None
        if not a.no_cpu and sample and D.world == 1:
            cpu = cpu_baselines(a, sample, want, a.level)
            if cpu["value"] is not None:
                cpu["gpu_over_cpu"] = {"vs_value": round(mbps / cpu["value"], 2),
                                       "vs_one_core": round(mbps / cpu["per_core_1thread"], 1),
                                       "vs_all_host_cpus_linear_estimate":
                                           round(mbps / cpu["all_host_cpus_linear_estimate"], 3)}
        line = {
            "metric": METRIC,
            "value": round(mbps, 1),
            "unit": "MB/s",
            "n_gpus": D.world,
            "steps": a.steps,
            "warmup": a.warmup,
            "ms_per_step": round(el / a.steps * 1e3, 2),
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "u8",
            "data": KIND_DATA[a.kind] if not a.cpu_dry_run else "cpu dry run: the generator's host twin (oracle/zgen.c), oracle",
            "config": {"workload": f"{KIND_CONFIG[a.kind]}: {a.buffers} x {a.buffer_bytes} B buffers per GPU, "
                                   f"deflate level {a.level}, zlib wrapper, inputs+outputs in HBM",
                       "level": a.level, "buffer_bytes": a.buffer_bytes,
                       "buffers_per_gpu": a.buffers, "inflight_mb": a.inflight_mb,
                       "parallelism": f"{D.world} GPU(s), one rank each, buffers sharded by index, "
                                      f"no data-path collective",
                       "collective_backend": D.backend, "world_size_seen": D.world},
            "compression_ratio": round(ratio, 4),
            "roofline": roof,
            "stage_ms_per_step": {k: round(v[0] / max(1, a.steps), 2) for k, v in st.items()},
            "crc32": None if crc is None else dict(crc, workload=f"C2: {a.crc_buffers} x {a.crc_bytes} B "
                                                                 f"uniform random per GPU"),
            "adler32": None if adl is None else dict(adl, workload=f"C5 shape: {a.adler_buffers} x "
                                                                   f"{a.adler_bytes} B small-vocabulary "
                                                                   f"text per GPU"),
            "inflate": None if inf is None else {
                "value": round(inf_total / inf_el / 1e6, 1), "unit": "MB/s (decompressed output)",
                "workload": "inflate of every stream the deflate leg wrote (zlib wrapper), outputs in HBM",
                "round_trip_bit_exact_all_buffers": True,
                "stage_ms_per_step": {"decode": round(inf["stages"]["parse_lazy"][0] / max(1, a.steps), 2),
                                      "match_copy": round(inf["stages"]["parse_greedy"][0] / max(1, a.steps), 2),
                                      "adler32": round(inf["stages"]["checksum"][0] / max(1, a.steps), 2),
                                      "finish": round(inf["stages"]["encode"][0] / max(1, a.steps), 2)}},
            "per_rank": [{"rank": r, "out_bytes": ob, "stream_crc_xor": "%08x" % (dg & 0xffffffff)}
                         for r, (dg, ob) in enumerate(digests)],
            "verified": {"deflate_buffers_bit_exact_vs_oracle": len(sample),
                         "deflate_buffers_bit_exact": shard_n,
                         "deflate_buffers_bit_exact_how": "every stream's length and device-computed CRC-32 "
                                                          "equal to the compiled reference's compress2() stream "
                                                          "(tests/golden/bench_shard_golden_r0.npz, " + shard_note
                                                          + ")" if shard_n else shard_note,
                         "per_rank_digest_vs_reference": shard_dig,
                         "crc32_values_checked": 0 if c is None else 64,
                         "adler32_values_checked": 0 if ad is None else min(2, ad["B"]),
                         "all_status_ok": True},
            "cpu_baseline": cpu,
            "memory_plan": memory_plan(a, D.world),
        }
        print(json.dumps(line), flush=True)
    D.close()


if __name__ == "__main__":
    main()
