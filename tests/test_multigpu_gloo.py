"""Multi-process (world size 2, gloo, CPU) coverage of the sharded path:
shard ranges, bitmap packing and the validity all-gather the GPU bench
runs over RCCL."""
import os
import socket

import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from tendermint_amd.shard import all_gather_validity, pack_bits, shard_range, unpack_bits


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, n, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    g = torch.Generator().manual_seed(1234)
    full = (torch.rand(n, generator=g) > 0.01).to(torch.uint8)  # same on every rank
    lo, hi = shard_range(n, world, rank)
    counts = [shard_range(n, world, r)[1] - shard_range(n, world, r)[0] for r in range(world)]
    got = all_gather_validity(full[lo:hi].clone(), counts)
    q.put((rank, bool(torch.equal(got, full))))
    dist.barrier()
    dist.destroy_process_group()


def test_shard_ranges_cover():
    for n in (0, 1, 7, 10_000, 10_001):
        for w in (1, 2, 3, 8):
            rs = [shard_range(n, w, r) for r in range(w)]
            assert rs[0][0] == 0 and rs[-1][1] == n
            assert all(rs[i][1] == rs[i + 1][0] for i in range(w - 1))
            assert max(b - a for a, b in rs) - min(b - a for a, b in rs) <= 1


def test_pack_unpack_roundtrip():
    for n in (1, 8, 9, 1000, 1003):
        v = (torch.rand(n) > 0.5).to(torch.uint8)
        assert torch.equal(unpack_bits(pack_bits(v), n), v)
        assert pack_bits(v).numel() == (n + 7) // 8


def test_all_gather_world2():
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, 10_001, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = [q.get(timeout=120) for _ in procs]
    for p in procs:
        p.join(timeout=60)
    assert sorted(res) == [(0, True), (1, True)]


def _status_worker(rank, world, port, q):
    """The bench's N > 1 exchange: each rank's contiguous int8 status vector
    of K batches (sr25519 Add errors are negative) gathered as one bitmap."""
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    K, n = 3, 1001
    g = torch.Generator().manual_seed(99 + rank)
    st = torch.randint(-2, 2, (K * n,), generator=g, dtype=torch.int8)
    got = all_gather_validity(st, [K * n] * world)
    mine = got[rank * K * n:(rank + 1) * K * n]
    q.put((rank, bool(torch.equal(mine, (st == 1).to(torch.uint8))), int(got.numel())))
    dist.barrier()
    dist.destroy_process_group()


def test_all_gather_statuses_world2():
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_status_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = sorted(q.get(timeout=120) for _ in procs)
    for p in procs:
        p.join(timeout=60)
    assert res == [(0, True, 6006), (1, True, 6006)]


def _sr_status_worker(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from tendermint_amd.shard import all_gather_statuses
    counts = [1001, 998]
    g = torch.Generator().manual_seed(7)
    full = torch.randint(-2, 2, (sum(counts),), generator=g, dtype=torch.int8)
    lo = sum(counts[:rank])
    got = all_gather_statuses(full[lo:lo + counts[rank]].clone(), counts)
    q.put((rank, bool(torch.equal(got, full)), int((got < 0).sum())))
    dist.barrier()
    dist.destroy_process_group()


def test_all_gather_sr25519_statuses_world2():
    """sr25519 Add-error statuses (-1 / -2) survive the gather
    (uneven shards)."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_sr_status_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = sorted(q.get(timeout=120) for _ in procs)
    for p in procs:
        p.join(timeout=60)
    assert [r[:2] for r in res] == [(0, True), (1, True)] and res[0][2] > 0


def test_bench_control_flow_world2():
    """bench.py's --gpus N path (one process per rank via torch.distributed.run,
    launches over streams, one validity all-gather per launch, barrier + MAX
    timing, rank 0's JSON line) executed with gloo and the --cpu-stub engine."""
    import json
    import subprocess
    import sys
    repo = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2", "--master-addr",
           "127.0.0.1", "--master-port", str(_free_port()), os.path.join(repo, "bench.py"), "--gpus", "2",
           "--steps", "7", "--warmup", "2", "--batch", "500", "--resident", "3", "--inflight", "2",
           "--batches-per-step", "3", "--cpu-stub", "--strong-n", "4003"]
    out = subprocess.run(cmd, capture_output=True, text=True, timeout=600, cwd=repo)
    assert out.returncode == 0, out.stderr[-3000:]
    lines = [ln for ln in out.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, out.stdout[-2000:]
    r = json.loads(lines[0])
    assert r["n_gpus"] == 2 and r["steps"] == 7 and r["warmup"] == 2 and r["value"] > 0
    # the rank count and backend the process group reported (a SCALE record shows them)
    assert r["config"]["parallelism"] == "shard2 (gloo, process group world size 2)"
    assert r["config"]["batches_per_step"] == 3
    assert r["run_timing"]["setup_s_max_over_ranks"] > 0
    # value = every rank's signatures: 2 ranks x 7 steps x 3 batches x 500
    assert abs(r["value"] * r["ms_per_step"] * 7e-3 / (2 * 7 * 3 * 500) - 1) < 1e-3
    assert "STUB" in r["data"]
    # the strong-scaling legs: one 4,003-signature batch (ed25519) and one
    # mixed batch split over both ranks, gathered and checked on every rank
    for leg in ("strong_1m", "strong_1m_mixed"):
        s = r[leg]
        assert s["signatures"] == 4003 and s["ranks"] == 2 and s["shard_per_rank"] == [2001, 2002]
        assert s["exact_vector_on_every_rank"] is True
        assert s["kernel_only"]["verifies_per_s"] > 0 and s["end_to_end"]["verifies_per_s"] > 0
    assert r["end_to_end_verifies_per_s"] > 0 and "end_to_end_vs_headline" in r
