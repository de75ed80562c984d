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
* cpu_baseline: the oracle port (oracle/liboracle.so, our C restatement of the
  reference deflate.c/trees.c) timed on this host's cores on a bounded sample of
  the same buffers; kind "port" (the compiled reference never leaves the build
  container); plus host system zlib on the same sample
  (`system_zlib`), checked byte-identical first.
* roofline.traffic: HBM bytes per launch from the committed rocprofv3 PMC
  passes of the same launch shape (profiles/), FETCH_SIZE x2 + WRITE_SIZE.
* After timing, a sample of outputs is checked bit-exact against the oracle and
  every status is checked.

Multi-GPU: launched by torch.distributed.run; buffers are sharded by global
index (rank r takes [r*B, (r+1)*B)), no data-path collective; one all_reduce
(max elapsed, sum bytes) at the end.
"""
import argparse
import concurrent.futures as cf
import ctypes as C
import json
import os
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
               "(40% text, 20% markup, 20% binary records, 10% random, 10% runs)",
    "enwik": "synthetic: device-generated seeded enwik-style 4 KiB segments (70% word text, 30% markup)",
    "vocab": "synthetic: device-generated seeded small-vocabulary text",
    "random": "synthetic: device-generated uniform random bytes",
}
KIND_CONFIG = {"silesia": "C4 per-GPU shard", "enwik": "C3-style", "vocab": "C5-style", "random": "random"}


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=3)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--buffers", type=int, default=int(os.environ.get("ZB_BUFFERS", 32768)),
                    help="1 MiB buffers per GPU (C4 shard = 32768)")
    ap.add_argument("--buffer-bytes", type=int, default=1 << 20)
    ap.add_argument("--level", type=int, default=6)
    ap.add_argument("--kind", default="silesia", choices=["random", "silesia", "enwik", "vocab"],
                    help="device generator: silesia (C4, default), enwik (C3), vocab (C5)")
    ap.add_argument("--crc-buffers", type=int, default=1 << 20)
    ap.add_argument("--crc-bytes", type=int, default=4096)
    ap.add_argument("--cpu-seconds", type=float, default=12.0)
    ap.add_argument("--cpu-threads", type=int, default=16)
    ap.add_argument("--no-cpu", action="store_true")
    ap.add_argument("--no-inflate", action="store_true", help="skip the inflate round-trip leg")
    ap.add_argument("--verify", type=int, default=8, help="outputs checked vs oracle")
    ap.add_argument("--inflight-mb", type=int, default=4096,
                    help="input bytes per deflate sub-batch (workspace ~15 B per byte)")
    return ap.parse_args()


def dist_setup():
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    torch.cuda.set_device(local)
    if world > 1:
        dist.init_process_group("nccl", device_id=torch.device("cuda", local))
    return world, rank


def barrier(world):
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()


def reduce_max(x, world):
    if world == 1:
        return x
    t = torch.tensor([x], dtype=torch.float64, device="cuda")
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item())


def reduce_sum(x, world):
    if world == 1:
        return x
    t = torch.tensor([x], dtype=torch.float64, device="cuda")
    dist.all_reduce(t, op=dist.ReduceOp.SUM)
    return float(t.item())


def shard(rank, world, per_gpu):
    """Global buffer indices owned by `rank`: a contiguous block of `per_gpu`
    (weak scaling: per-GPU work is fixed, the job grows with N)."""
    return rank * per_gpu, (rank + 1) * per_gpu


def deflate_leg(a, world, rank):
    n, B = a.buffer_bytes, a.buffers
    first, _ = shard(rank, world, B)
    cap = (zgpu.compress_bound(n) + 15) // 16 * 16
    src = torch.empty(n * B, dtype=torch.uint8, device="cuda")
    kind = {"random": 0, "silesia": 1, "enwik": 2, "vocab": 3}[a.kind]
    zgpu.generate_dev(src, n, B, kind, seed=2025, first_index=first)
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
    barrier(world)
    zgpu.stage_timing(True)
    t0 = time.perf_counter()
    for _ in range(a.steps):
        step()
    barrier(world)
    el = time.perf_counter() - t0
    zgpu.stage_timing(False)
    stages = zgpu.stage_timing_read()
    sts = st.cpu()
    assert int((sts != 0).sum()) == 0, "deflate status != Z_OK"
    out_bytes = int(dlen.sum().item())
    return dict(src=src, dst=dst, dlen=dlen, cap=cap, elapsed=el, stages=stages,
                out_bytes=out_bytes, in_bytes=n * B)


def crc_leg(a, world, rank):
    n, B = a.crc_bytes, a.crc_buffers
    first, _ = shard(rank, world, B)
    src = torch.empty(n * B, dtype=torch.uint8, device="cuda")
    zgpu.generate_dev(src, n, B, zgpu.KIND_RANDOM, seed=77, first_index=first)
    off = torch.arange(B, dtype=torch.int64, device="cuda") * n
    ln = torch.full((B,), n, dtype=torch.int64, device="cuda")
    out = torch.zeros(B, dtype=torch.int32, device="cuda")
    stream = torch.cuda.current_stream()
    for _ in range(max(1, a.warmup)):
        zgpu.crc32_batch_dev(src, off, ln, out)
    barrier(world)
    evs = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
           for _ in range(a.steps)]
    t0 = time.perf_counter()
    for e0, e1 in evs:
        e0.record(stream)
        zgpu.crc32_batch_dev(src, off, ln, out)
        e1.record(stream)
    barrier(world)
    el = time.perf_counter() - t0
    kms = sum(e0.elapsed_time(e1) for e0, e1 in evs) / len(evs)
    return dict(src=src, out=out, elapsed=el, kernel_ms=kms, bytes=n * B)


def inflate_leg(a, world, d):
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
    barrier(world)
    zgpu.stage_timing(True)
    t0 = time.perf_counter()
    for _ in range(a.steps):
        step()
    barrier(world)
    el = time.perf_counter() - t0
    zgpu.stage_timing(False)
    stages = zgpu.stage_timing_read()
    ok = int((ost != 0).sum().item()) == 0 and bool((olen == n).all().item()) and bool(torch.equal(out, src))
    assert ok, "inflate(deflate(x)) != x on the device"
    del out
    return dict(elapsed=el, stages=stages, out_bytes=n * B, in_bytes=int(dlen.sum().item()))


def launches_tag(a):
    """Shape of one deflate launch (sub-batch): buffers x bytes."""
    per = max(1, min(a.buffers, (a.inflight_mb << 20) // a.buffer_bytes))
    return f"{per}x{a.buffer_bytes}"


def cpu_baseline(a, sample, level):
    """Oracle port timed on host cores over a bounded, repeated sample."""
    from zhelpers import Oracle
    o = Oracle()
    threads = max(1, min(a.cpu_threads, os.cpu_count() or 1))
    deadline = time.perf_counter() + a.cpu_seconds

    def work(tid):
        done, k = 0, tid
        while time.perf_counter() < deadline:
            b = sample[k % len(sample)]
            o.compress(b, level)
            done += len(b)
            k += threads
        return done

    t0 = time.perf_counter()
    with cf.ThreadPoolExecutor(threads) as ex:
        total = sum(ex.map(work, range(threads)))
    el = time.perf_counter() - t0
    return total / el / 1e6, threads, total


def system_zlib_baseline(a, sample, level, want):
    """Host zlib (Python's zlib module: the system libz, GIL released) on the
    same sample; its output is checked against the GPU streams first."""
    import zlib
    for b, z in zip(sample, want):
        if zlib.compress(b, level) != z:
            return {"value": None, "version": zlib.ZLIB_RUNTIME_VERSION,
                    "note": "system zlib output differs from the reference stream; not timed"}
    threads = max(1, min(a.cpu_threads, os.cpu_count() or 1))
    deadline = time.perf_counter() + a.cpu_seconds

    def work(tid):
        done, k = 0, tid
        while time.perf_counter() < deadline:
            b = sample[k % len(sample)]
            zlib.compress(b, level)
            done += len(b)
            k += threads
        return done

    t0 = time.perf_counter()
    with cf.ThreadPoolExecutor(threads) as ex:
        total = sum(ex.map(work, range(threads)))
    el = time.perf_counter() - t0
    return {"value": round(total / el / 1e6, 2), "unit": "MB/s", "cores": threads,
            "version": zlib.ZLIB_RUNTIME_VERSION, "bit_identical_on_sample": True,
            "sample": f"same {len(sample)} buffers, ~{a.cpu_seconds:.0f} s, {total / 1e6:.0f} MB"}


def pmc_traffic(kernel, launch_bytes_hint):
    """HBM bytes per launch of `kernel` from the committed rocprofv3 PMC passes
    (profiles/*_pmc_fetch_*.csv, *_pmc_write_*.csv; FETCH_SIZE doubled per the
    gfx950 streaming-read correction, units KiB).  Only for profiles taken on
    this launch's shape (file name carries the shape tag)."""
    import csv
    import glob
    tag = launch_bytes_hint
    fetch = sorted(glob.glob(os.path.join(ROOT, "profiles", f"*_pmc_fetch_*{tag}*.csv")))
    write = sorted(glob.glob(os.path.join(ROOT, "profiles", f"*_pmc_write_*{tag}*.csv")))
    if not fetch or not write:
        return None, None

    def per_launch(path, counter):
        vals = [float(r["Counter_Value"]) for r in csv.DictReader(open(path))
                if r["Counter_Name"] == counter and kernel in r["Kernel_Name"]]
        return sum(vals) / len(vals) * 1024.0 if vals else None

    f = per_launch(fetch[-1], "FETCH_SIZE")
    w = per_launch(write[-1], "WRITE_SIZE")
    if f is None or w is None:
        return None, None
    return 2.0 * f + w, os.path.basename(fetch[-1]) + " + " + os.path.basename(write[-1])


def main():
    a = parse()
    world, rank = dist_setup()
    zgpu.load()
    assert zgpu.load().zgpu_init() == 0, "libzgpu: GPU init failed"
    zgpu.set_inflight_bytes(a.inflight_mb << 20)

    d = deflate_leg(a, world, rank)
    inf = None if a.no_inflate else inflate_leg(a, world, d)
    c = crc_leg(a, world, rank)

    # ---- verification (outside the timed region) ----
    from zhelpers import Oracle
    o = Oracle()
    h_dlen = d["dlen"].cpu().numpy()
    n = a.buffer_bytes
    idx = sorted(set(int(i) for i in torch.linspace(0, a.buffers - 1, a.verify).tolist())) if a.verify > 0 else []
    sample, want = [], []
    for i in idx:
        raw = d["src"][i * n:(i + 1) * n].cpu().numpy().tobytes()
        z = d["dst"][i * d["cap"]: i * d["cap"] + int(h_dlen[i])].cpu().numpy().tobytes()
        assert z == o.compress(raw, a.level)[1], f"buffer {i}: GPU stream != oracle"
        sample.append(raw)
        want.append(z)
    crc_h = c["out"][:64].cpu().numpy().view("uint32")
    for i in range(64):
        raw = c["src"][i * a.crc_bytes:(i + 1) * a.crc_bytes].cpu().numpy().tobytes()
        assert int(crc_h[i]) == o.crc32(raw), f"crc buffer {i} mismatch"

    el = reduce_max(d["elapsed"], world)
    in_total = reduce_sum(float(d["in_bytes"]) * a.steps, world)
    out_total = reduce_sum(float(d["out_bytes"]), world)
    if inf is not None:
        inf_el = reduce_max(inf["elapsed"], world)
        inf_total = reduce_sum(float(inf["out_bytes"]) * a.steps, world)
    crc_el = reduce_max(c["elapsed"], world)
    crc_total = reduce_sum(float(c["bytes"]) * a.steps, world)

    if rank == 0:
        mbps = in_total / el / 1e6
        ratio = (d["in_bytes"]) / max(1, d["out_bytes"])
        st = d["stages"]
        # dominant kernel: k_match ("match"); algorithmic bytes per launch =
        # Σ (n + out_len) over the buffers one launch processes
        mms, mcount = st["match"]
        per_step_alg = d["in_bytes"] + d["out_bytes"]
        launches_per_step = max(1, mcount // max(1, a.steps))
        alg_per_launch = per_step_alg / launches_per_step
        m_avg_ms = mms / max(1, mcount)
        achieved = alg_per_launch / (m_avg_ms / 1e3) / 1e9 if m_avg_ms > 0 else 0.0
        crc_alg = (a.crc_bytes + 4) * a.crc_buffers
        crc_gbs_kernel = crc_alg / (c["kernel_ms"] / 1e3) / 1e9
        cpu = None
        m_traffic, m_src = pmc_traffic("k_match", f"L{a.level}_{launches_tag(a)}")
        c_traffic, c_src = pmc_traffic("k_crc32", f"C2_{a.crc_buffers}x{a.crc_bytes}")
        if not a.no_cpu and sample:
            v, threads, tot = cpu_baseline(a, sample, a.level)
            cpu = {"value": round(v, 2), "unit": "MB/s", "cores": threads, "kind": "port",
                   "sample": f"{len(sample)} distinct 1 MiB {a.kind} buffers of this batch, "
                             f"compressed repeatedly at level {a.level} for ~{a.cpu_seconds:.0f} s "
                             f"({tot / 1e6:.0f} MB) by oracle/liboracle.so on {threads} host threads",
                   "system_zlib": system_zlib_baseline(a, sample, a.level, want)}
        line = {
            "metric": METRIC,
            "value": round(mbps, 1),
            "unit": "MB/s",
            "n_gpus": world,
            "steps": a.steps,
            "warmup": a.warmup,
            "ms_per_step": round(el / a.steps * 1e3, 2),
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "u8",
            "data": KIND_DATA[a.kind],
            "config": {"workload": f"{KIND_CONFIG[a.kind]}: {a.buffers} x {a.buffer_bytes} B buffers, "
                                   f"deflate level {a.level}, zlib wrapper, inputs+outputs in HBM",
                       "level": a.level, "buffer_bytes": a.buffer_bytes,
                       "buffers_per_gpu": a.buffers, "inflight_mb": a.inflight_mb,
                       "parallelism": f"{world} GPU(s), buffers sharded by index, no data-path collective"},
            "compression_ratio": round(ratio, 4),
            "roofline": {"bound": "hbm", "kernel": "k_match",
                         "achieved": round(achieved, 2), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                         "frac": round(achieved / HBM_PEAK_GBS, 6),
                         "traffic": None if m_traffic is None else int(m_traffic),
                         "traffic_source": m_src,
                         "alg_bytes_per_launch": int(alg_per_launch),
                         "avg_launch_ms": round(m_avg_ms, 3),
                         "limiter": "not HBM: dependent LDS round trips of the chain walks and instruction "
                                    "issue at the 16 waves/CU the 148.5 KiB LDS window allows (DESIGN.md 4.3)"},
            "stage_ms_per_step": {k: round(v[0] / max(1, a.steps), 2) for k, v in st.items()},
            "crc32": {"value": round(crc_total / crc_el / 1e9, 2), "unit": "GB/s",
                      "workload": f"C2: {a.crc_buffers} x {a.crc_bytes} B uniform random per GPU",
                      "roofline": {"bound": "hbm", "kernel": "k_crc32",
                                   "achieved": round(crc_gbs_kernel, 1), "peak": HBM_PEAK_GBS,
                                   "unit": "GB/s", "frac": round(crc_gbs_kernel / HBM_PEAK_GBS, 4),
                                   "traffic": None if c_traffic is None else int(c_traffic),
                                   "traffic_source": c_src,
                                   "alg_bytes_per_launch": crc_alg,
                                   "avg_launch_ms": round(c["kernel_ms"], 4)}},
            "inflate": None if inf is None else {
                "value": round(inf_total / inf_el / 1e6, 1), "unit": "MB/s (decompressed output)",
                "workload": "inflate of every stream the deflate leg wrote (zlib wrapper), outputs in HBM",
                "round_trip_bit_exact_all_buffers": True,
                "stage_ms_per_step": {"decode": round(inf["stages"]["parse_lazy"][0] / max(1, a.steps), 2),
                                      "match_copy": round(inf["stages"]["parse_greedy"][0] / max(1, a.steps), 2),
                                      "adler32": round(inf["stages"]["checksum"][0] / max(1, a.steps), 2),
                                      "finish": round(inf["stages"]["encode"][0] / max(1, a.steps), 2)}},
            "verified": {"deflate_buffers_bit_exact_vs_oracle": len(sample),
                         "crc32_values_checked": 64, "all_status_ok": True},
            "cpu_baseline": cpu,
        }
        print(json.dumps(line), flush=True)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
