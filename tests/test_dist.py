"""Multi-process (gloo, CPU) test of the benchmark's multi-GPU decomposition:
buffers are sharded by global index with no data-path collective, and the
only collectives are the final max(elapsed) / sum(bytes) reductions.  Compute
is done with the oracle on tiny inputs (no GPU here)."""
import os
import socket

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

import datagen


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def _worker(rank, world, port, per_gpu, q):
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    sys.path.insert(0, root)
    sys.path.insert(0, os.path.join(root, "tests"))
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    import bench
    from zhelpers import Oracle
    o = Oracle()
    lo, hi = bench.shard(rank, world, per_gpu)
    in_bytes = out_bytes = 0
    crcs = []
    for gidx in range(lo, hi):
        data = datagen.mix(3000 + 17 * gidx, gidx)
        z = o.compress(data, 6)[1]
        in_bytes += len(data)
        out_bytes += len(z)
        crcs.append(o.crc32(z))
    t = torch.tensor([float(in_bytes), float(out_bytes)], dtype=torch.float64)
    dist.all_reduce(t, op=dist.ReduceOp.SUM)
    el = torch.tensor([0.1 * (rank + 1)], dtype=torch.float64)
    dist.all_reduce(el, op=dist.ReduceOp.MAX)
    gathered = [None] * world
    dist.all_gather_object(gathered, (lo, hi, crcs))
    if rank == 0:
        q.put((t.tolist(), float(el.item()), gathered))
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("world", [2])
def test_sharded_batch_matches_single_process(world):
    per_gpu = 5
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, per_gpu, q)) for r in range(world)]
    for p in procs:
        p.start()
    (tot_in, tot_out), el, gathered = q.get(timeout=240)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    # shards are disjoint and cover [0, world*per_gpu)
    idx = sorted(i for lo, hi, _ in gathered for i in range(lo, hi))
    assert idx == list(range(world * per_gpu))
    # aggregate equals a single-process pass over the same global batch
    from zhelpers import Oracle
    o = Oracle()
    want_in = want_out = 0
    want_crc = []
    for gidx in range(world * per_gpu):
        data = datagen.mix(3000 + 17 * gidx, gidx)
        z = o.compress(data, 6)[1]
        want_in += len(data)
        want_out += len(z)
        want_crc.append(o.crc32(z))
    assert (tot_in, tot_out) == (want_in, want_out)
    assert [c for _, _, cs in gathered for c in cs] == want_crc
    assert abs(el - 0.1 * world) < 1e-9


def test_bench_gpus_flag_launches_ranks():
    """`bench.py --gpus 2` (no launcher in the environment) must start 2 ranks
    itself and report n_gpus == 2 with the collectives' aggregate: a run that
    ignored --gpus would print n_gpus 1 and only rank 0's bytes."""
    import json
    import subprocess
    import sys
    import zlib
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    env = {k: v for k, v in os.environ.items()
           if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT")}
    per_gpu, nbytes = 3, 20000
    r = subprocess.run([sys.executable, os.path.join(root, "bench.py"), "--gpus", "2", "--cpu-dry-run",
                        "--buffers", str(per_gpu), "--buffer-bytes", str(nbytes), "--steps", "1",
                        "--warmup", "0"], capture_output=True, text=True, timeout=300, env=env, cwd="/tmp")
    assert r.returncode == 0, r.stderr[-2000:]
    line = json.loads([s for s in r.stdout.splitlines() if s.startswith("{")][-1])
    assert line["n_gpus"] == 2 and line["config"]["world_size_seen"] == 2
    assert line["config"]["collective_backend"] == "gloo"
    from zhelpers import Oracle
    o = Oracle()
    for rank, pr in enumerate(line["per_rank"]):
        ob, dg = 0, 0
        for g in range(rank * per_gpu, (rank + 1) * per_gpu):
            z = o.compress(o.generate(nbytes, 1, 1, 2025, g)[0], 6)[1]
            ob += len(z)
            dg ^= zlib.crc32(z)
        assert pr["out_bytes"] == ob and pr["stream_crc_xor"] == "%08x" % dg
    want_ratio = 2 * per_gpu * nbytes / sum(p["out_bytes"] for p in line["per_rank"])
    assert abs(line["compression_ratio"] - want_ratio) < 1e-3


def test_bench_rejects_mismatched_world():
    """Under a launcher, --gpus must equal WORLD_SIZE (no silent 1-GPU run)."""
    import subprocess
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    env = dict(os.environ, WORLD_SIZE="1", RANK="0", LOCAL_RANK="0")
    r = subprocess.run([sys.executable, os.path.join(root, "bench.py"), "--gpus", "4", "--cpu-dry-run",
                        "--buffers", "1", "--buffer-bytes", "1000"], capture_output=True, text=True,
                       timeout=120, env=env)
    assert r.returncode != 0 and "WORLD_SIZE=1" in (r.stderr + r.stdout)


def test_bench_world8_dry_run_matches_reference_digests():
    """`bench.py --gpus 8 --cpu-dry-run` at a small size: eight gloo ranks
    (launched by bench.py itself), each compressing its shard of the Silesia-
    style generator's buffers, reduce and all_gather exactly as on eight GPUs;
    every rank's digest (sum of stream lengths, XOR of stream CRC-32s) must equal
    the compiled reference's for the same global indices
    (tests/golden/bench_shard_golden_small.json, make_bench_shard_golden_small.py)."""
    import json
    import subprocess
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    g = json.load(open(os.path.join(root, "tests", "golden", "bench_shard_golden_small.json")))
    env = {k: v for k, v in os.environ.items()
           if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT")}
    env["OMP_NUM_THREADS"] = "1"
    r = subprocess.run([sys.executable, os.path.join(root, "bench.py"), "--gpus", "8", "--cpu-dry-run",
                        "--buffers", str(g["buffers_per_rank"]), "--buffer-bytes", str(g["buffer_bytes"]),
                        "--steps", "1", "--warmup", "0"], capture_output=True, text=True, timeout=600, env=env,
                       cwd="/tmp")
    assert r.returncode == 0, r.stderr[-2000:]
    line = json.loads([s for s in r.stdout.splitlines() if s.startswith("{")][-1])
    assert line["n_gpus"] == 8 and line["config"]["world_size_seen"] == 8
    assert line["config"]["collective_backend"] == "gloo"
    assert [p["rank"] for p in line["per_rank"]] == list(range(8))
    for pr in line["per_rank"]:
        want = g["ranks"][str(pr["rank"])]
        assert {"out_bytes": pr["out_bytes"], "stream_crc_xor": pr["stream_crc_xor"]} == want, pr
    assert line["verified"]["per_rank_digest_vs_reference"] is True
    total_in = 8 * g["buffers_per_rank"] * g["buffer_bytes"]
    assert abs(line["compression_ratio"] - total_in / sum(w["out_bytes"] for w in g["ranks"].values())) < 1e-3
    assert line["memory_plan"]["hbm_fits"] is True


def test_bench_memory_plan_per_rank():
    """`bench.py --gpus 8 --plan-only`: the HBM each rank of the default C4 run
    holds -- 32 GiB in, 32 GiB out, ~31 B of deflate workspace per in-flight
    byte (4 GiB), the inflate leg's output and records, the checksum legs'
    inputs -- must fit an MI355X's 288 GB, and the host side must fit the
    host; a sub-batch budget twice as large must be reported as not fitting."""
    import json
    import subprocess
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

    def plan(*extra):
        r = subprocess.run([sys.executable, os.path.join(root, "bench.py"), "--gpus", "8", "--plan-only", *extra],
                           capture_output=True, text=True, timeout=120)
        assert r.returncode == 0, r.stderr[-2000:]
        return json.loads(r.stdout.strip().splitlines()[-1])["memory_plan"]

    p = plan()
    legs = p["hbm_bytes_per_rank"]
    assert legs["deflate_inputs"] == 32768 << 20
    assert 30 * (4 << 30) < legs["deflate_workspace"] < 36 * (4 << 30)
    assert p["hbm_need_per_rank"] == sum(legs.values())
    assert p["hbm_fits"] is True and p["hbm_need_per_rank"] <= 288e9
    assert p["host_need_all_ranks_est"] == 8 * p["host_bytes_per_rank_est"]
    assert plan("--inflight-mb", "8192")["hbm_fits"] is False
