"""Multi-rank path on CPU (gloo, world_size 2): the batch sharding that
bench.py uses for the 1/2/4/8-GPU curve (batch x head split,
no collective on the data path).  Each rank computes its shard with the oracle;
the concatenated shards must equal the unsharded result bit-for-bit, and the
max-over-ranks timing reduction must pick the slowest rank."""
import os
import socket

import numpy as np
import pytest

torch = pytest.importorskip("torch")
import torch.distributed as dist  # noqa: E402
import torch.multiprocessing as mp  # noqa: E402

import bench  # noqa: E402


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def test_shard_range_partitions():
    for total in (1, 2, 5, 8, 63, 64):
        for world in (1, 2, 3, 4, 8):
            spans = [bench.shard_range(total, world, r) for r in range(world)]
            assert spans[0][0] == 0 and spans[-1][1] == total
            for (a, b), (c, d) in zip(spans, spans[1:]):
                assert b == c
            sizes = [b - a for a, b in spans]
            assert max(sizes) - min(sizes) <= 1


def test_flop_and_byte_conventions():
    # reference convention: 4*B*H*S^2*D, halved when causal (flash_attention.cu:938-939)
    assert bench.attention_flops(1, 32, 8192, 128, False) == 4 * 32 * 8192 ** 2 * 128
    assert bench.attention_flops(64, 32, 4096, 128, True) == 2 * 64 * 32 * 4096 ** 2 * 128
    assert bench.algorithmic_bytes(1, 32, 1024, 128) == 8 * 32 * 1024 * 128
    assert abs(bench.mfma_peak_tflops(256) - 2516.58) < 0.1


def _worker(rank, world, port, result_q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    import oracle

    B, H, S = 5, 2, 48
    q, k, v = oracle.gen_inputs(B, H, S, 128, 42)
    lo, hi = bench.shard_range(B, world, rank)
    o_local = oracle.attention(q[lo:hi], k[lo:hi], v[lo:hi], True, threads=1)
    # gather variable-size shards (pad to the max shard) -- verification only
    maxb = max(bench.shard_range(B, world, r)[1] - bench.shard_range(B, world, r)[0]
               for r in range(world))
    buf = np.zeros((maxb, H, S, 128), np.int32)  # gloo has no 16-bit integer type
    buf[: hi - lo] = o_local
    t = torch.from_numpy(buf)
    parts = [torch.zeros_like(t) for _ in range(world)]
    dist.all_gather(parts, t)
    # max-over-ranks timing reduction, as bench.py does
    el = torch.tensor([1.0 + rank], dtype=torch.float64)
    dist.all_reduce(el, op=dist.ReduceOp.MAX)
    if rank == 0:
        shards = []
        for r in range(world):
            a, b = bench.shard_range(B, world, r)
            shards.append(parts[r].numpy()[: b - a].astype(np.uint16))
        got = np.concatenate(shards)
        ref = oracle.attention(q, k, v, True, threads=1)
        result_q.put((bool(np.array_equal(got, ref)), float(el.item())))
    dist.barrier()
    dist.destroy_process_group()


def test_batch_sharded_oracle_world2():
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.SimpleQueue()
    mp.start_processes(_worker, args=(world, _free_port(), q), nprocs=world, join=True,
                       start_method="spawn")
    equal, el = q.get()
    assert equal, "concatenated batch shards differ from the unsharded oracle"
    assert el == float(world)  # max over ranks of (1 + rank)
