"""Multi-process (gloo, world_size 2) tests of the parallel layer - no cluster needed.

* object all_gather / reduce_tensor (reference ddp_utils.py)
* GradReducer: W=2 half batches == W=1 full batch gradients (DDP equivalence),
  with SyncBN (cross-replica statistics) so BN layers see the global batch
* SyncBN forward/backward == single-process BN on the concatenated batch
* parameter broadcast at construction (DDP's _sync_module_states)
"""
import os
import socket

import pytest
import torch
import torch.multiprocessing as mp


def _port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _setup(rank, world, port):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank),
                      WORLD_SIZE=str(world), LOCAL_RANK=str(rank))
    from pytorch_imageclassification_distributed_amd.parallel import init_distributed
    return init_distributed(device="cpu", backend="gloo")


def _run(fn, world=2):
    port = _port()
    mp.spawn(fn, args=(world, port), nprocs=world, join=True)


# ---------------------------------------------------------------------------
def _w_comm(rank, world, port):
    ctx = _setup(rank, world, port)
    import ddp_utils
    out = ddp_utils.all_gather({"rank": rank, "pad": "x" * (10 + 50 * rank)})
    assert [o["rank"] for o in out] == [0, 1] and len(out[1]["pad"]) == 60
    t = ddp_utils.reduce_tensor(torch.tensor([float(rank + 1)]))
    assert t.item() == pytest.approx(1.5)
    from pytorch_imageclassification_distributed_amd.parallel import all_gather_tensor
    g = all_gather_tensor(torch.tensor([rank, 10 + rank]))
    assert g.tolist() == [[0, 10], [1, 11]]
    assert ctx.world_size == 2


def test_object_all_gather_and_reduce():
    _run(_w_comm)


# ---------------------------------------------------------------------------
def _model(seed):
    from pytorch_imageclassification_distributed_amd.models import Classifier
    torch.manual_seed(seed)
    return Classifier("resnet18", 4)


def _w_ddp(rank, world, port):
    _setup(rank, world, port)
    import torch.nn.functional as F
    from pytorch_imageclassification_distributed_amd.parallel import GradReducer, convert_sync_batchnorm
    torch.manual_seed(123)
    x = torch.randn(8, 3, 16, 16)
    y = torch.randint(0, 4, (8,))
    # reference: one process, full batch, plain BN
    ref = _model(0)
    F.cross_entropy(ref(x), y).backward()
    # distributed: different init on rank 1 (must be overwritten by the broadcast)
    m = _model(rank)
    convert_sync_batchnorm(m)
    red = GradReducer(m, bucket_cap_mb=0.5, first_bucket_mb=0.1)
    assert len(red.buckets) > 2
    for it in range(2):  # second iteration runs on the rebuilt bucket layout
        for p in m.parameters():
            p.grad = None
        xs, ys = x[rank * 4:(rank + 1) * 4], y[rank * 4:(rank + 1) * 4]
        F.cross_entropy(m(xs), ys).backward()
        scale = red.finish()
    for (n, p), (_n, q) in zip(m.named_parameters(), ref.named_parameters()):
        assert torch.allclose(p.grad * scale, q.grad, rtol=1e-4, atol=1e-5), n


def test_grad_reducer_matches_single_process():
    _run(_w_ddp)


def _w_flat_dtype(rank, world, port):
    """The post-replay flat all-reduce (``deferred`` capture at N > 1) moves the gradients in the same transport
    dtype as the bucketed path: with --comm-dtype bf16 both give bitwise the same reduced gradients."""
    _setup(rank, world, port)
    import torch.nn.functional as F
    from pytorch_imageclassification_distributed_amd.parallel import GradReducer
    torch.manual_seed(5)
    x, y = torch.randn(8, 3, 16, 16), torch.randint(0, 4, (8,))
    xs, ys = x[rank * 4:(rank + 1) * 4], y[rank * 4:(rank + 1) * 4]
    out = {}
    for mode in ("bucketed", "flat"):
        m = _model(0)
        red = GradReducer(m, bucket_cap_mb=0.5, first_bucket_mb=0.1, comm_dtype=torch.bfloat16,
                          rebuild_buckets=False)
        red.deferred = mode == "flat"
        F.cross_entropy(m(xs), ys).backward()
        red.finish() if mode == "bucketed" else red.flat_all_reduce()
        out[mode] = red.flat.clone()
        red.remove_hooks()
    assert torch.equal(out["bucketed"], out["flat"])
    assert torch.equal(out["flat"], out["flat"].to(torch.bfloat16).float())  # really moved as bf16


def test_flat_all_reduce_honours_comm_dtype():
    _run(_w_flat_dtype)


def test_resnet50_bucket_plan_bounds_the_tail():
    """The ResNet-50 bucket plan (VERDICT r4 next #5a): 1 MiB first bucket, <= 32 MiB buckets, and the last
    bucket - layer1 + stem, the gradients backward produces last, ~28 MiB as one bucket - cut into <= 4 MiB
    pieces, so only the final piece's all-reduce is left after the weight-gradient side stream drains."""
    from pytorch_imageclassification_distributed_amd.models import Classifier
    from pytorch_imageclassification_distributed_amd.parallel import GradReducer
    m = Classifier("resnet50", 7)
    whole = GradReducer(m, bucket_cap_mb=32.0, tail_bucket_mb=0)
    cut = GradReducer(m, bucket_cap_mb=32.0, tail_bucket_mb=4.0)
    a, b = whole.bucket_sizes_mb(), cut.bucket_sizes_mb()
    assert a[0] <= 1.0 and all(v <= 32.0 for v in a) and a[-1] > 20.0  # the unbounded tail bucket
    assert b[:len(a) - 1] == a[:-1]  # only the last bucket changes
    tail = b[len(a) - 1:]
    assert len(tail) >= 6 and all(v <= 4.0 for v in tail) and abs(sum(tail) - a[-1]) < 1e-6
    # contiguous cover of the flat buffer, in ready order; the stem conv's gradient is in the very last piece
    assert cut.buckets[0][0] == 0 and cut.buckets[-1][1] == cut.flat.numel()
    assert all(x[1] == y[0] for x, y in zip(cut.buckets, cut.buckets[1:]))
    stem = cut.index[id(m.encoder.conv1.weight)]
    assert cut.bucket_of[stem] == len(cut.buckets) - 1
    for r in (whole, cut):
        r.remove_hooks()


# ---------------------------------------------------------------------------
def _w_syncbn(rank, world, port):
    _setup(rank, world, port)
    import torch.nn as nn
    from pytorch_imageclassification_distributed_amd.parallel import sync_batch_norm
    import torch.distributed as dist
    torch.manual_seed(7)
    x = torch.randn(6, 5, 4, 4) * 3 + 1
    gy = torch.randn(6, 5, 4, 4)
    bn_ref = nn.BatchNorm2d(5)
    xr = x.clone().requires_grad_(True)
    yr = bn_ref(xr)
    yr.backward(gy)
    bn = nn.BatchNorm2d(5)
    sl = slice(0, 2) if rank == 0 else slice(2, 6)  # unequal per-rank counts
    xs = x[sl].clone().requires_grad_(True)
    ys = sync_batch_norm(xs, bn, dist.group.WORLD)
    assert torch.allclose(ys, yr[sl], atol=1e-5)
    ys.backward(gy[sl])
    assert torch.allclose(xs.grad, xr.grad[sl], atol=1e-5)
    assert torch.allclose(bn.running_mean, bn_ref.running_mean, atol=1e-6)
    assert torch.allclose(bn.running_var, bn_ref.running_var, atol=1e-5)
    gw = bn.weight.grad.clone()
    dist.all_reduce(gw)
    assert torch.allclose(gw, bn_ref.weight.grad, atol=1e-4)


def test_syncbn_matches_global_batch_norm():
    _run(_w_syncbn)


# ---------------------------------------------------------------------------
def _w_train(rank, world, port):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank),
                      WORLD_SIZE=str(world), LOCAL_RANK=str(rank))
    import train
    ck = os.environ["_TEST_CKPT"]
    hist = train.main(["--synthetic", "--model", "resnet18", "--image-size", "16", "--device", "cpu",
                       "--batchsize", "8", "--epochs", "2", "--num-workers", "0", "--synthetic-train-size", "64",
                       "--synthetic-val-size", "16", "--ckpt-dir", ck, "--lr", "1e-3", "--no-progress",
                       "--val-batchsize", "4", "--resume", "none"])
    assert len(hist) == 2
    import json
    with open(os.path.join(ck, f"hist{rank}.json"), "w") as f:
        json.dump(hist, f)


def test_train_cli_two_processes(tmp_path):
    os.environ["_TEST_CKPT"] = str(tmp_path)
    _run(_w_train)
    import json
    h0 = json.load(open(tmp_path / "hist0.json"))
    h1 = json.load(open(tmp_path / "hist1.json"))
    assert [r["val_acc"] for r in h0] == [r["val_acc"] for r in h1]  # combined accuracy on all ranks
    assert [r["train_loss"] for r in h0] == pytest.approx([r["train_loss"] for r in h1])  # globally averaged loss
    assert (tmp_path / "resnet18" / "best_model").exists()


# ---------------------------------------------------------------------------
def _w_fault(rank, world, port, marker, timeout_min):
    import time
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank),
                      WORLD_SIZE=str(world), LOCAL_RANK=str(rank))
    import torch.distributed as dist
    from pytorch_imageclassification_distributed_amd.parallel import init_distributed
    init_distributed(device="cpu", backend="gloo", timeout_min=timeout_min)
    dist.barrier()
    if rank == 1:
        os._exit(17)  # injected fault: the rank disappears without a clean shutdown
    t0 = time.time()
    try:
        for _ in range(1000):
            dist.all_reduce(torch.ones(1024))
            time.sleep(0.01)
        outcome = "no-error"
    except Exception as e:  # noqa: BLE001 - any collective error is the expected outcome
        outcome = type(e).__name__
    with open(marker, "w") as f:
        f.write(f"{outcome} {time.time() - t0:.2f}")
    os._exit(0)


def test_rank_failure_is_detected(tmp_path):
    """Fault injection: when a peer dies mid-run the surviving rank's collective fails
    within the process-group timeout instead of hanging."""
    ctxm = mp.get_context("spawn")
    port, marker = _port(), str(tmp_path / "rank0.txt")
    procs = [ctxm.Process(target=_w_fault, args=(r, 2, port, marker, 0.5)) for r in range(2)]
    for p_ in procs:
        p_.start()
    for p_ in procs:
        p_.join(timeout=120)
    alive = [p_ for p_ in procs if p_.is_alive()]
    for p_ in alive:
        p_.kill()
    assert not alive, "a rank hung after its peer died"
    outcome, secs = open(marker).read().split()
    assert outcome != "no-error"
    assert float(secs) < 60


def _w_buffers(rank, world, port):
    _setup(rank, world, port)
    import torch.nn as nn
    from pytorch_imageclassification_distributed_amd.parallel import GradReducer
    m = nn.Sequential(nn.Conv2d(3, 4, 1), nn.BatchNorm2d(4))
    torch.manual_seed(0)
    for p_ in m.parameters():
        nn.init.normal_(p_)
    red = GradReducer(m, broadcast=False)
    m[1].running_mean.fill_(float(rank + 1))
    m[1].num_batches_tracked.fill_(rank + 5)
    red.sync_buffers()
    assert torch.all(m[1].running_mean == 1.0) and int(m[1].num_batches_tracked) == 5


def test_broadcast_buffers():
    """DDP broadcast_buffers parity (X3): rank 0's BN buffers overwrite the other ranks'."""
    _run(_w_buffers)


# ---------------------------------------------------------------------------
def _w_shapes(rank, world, port):
    _setup(rank, world, port)
    from pytorch_imageclassification_distributed_amd.models import Classifier
    from pytorch_imageclassification_distributed_amd.parallel import GradReducer
    m = Classifier("resnet18", 4 if rank == 0 else 5)  # head differs on rank 1
    with pytest.raises(RuntimeError, match="parameter list differs"):
        GradReducer(m)


def test_grad_reducer_verifies_param_shapes():
    """X1: DDP's _verify_param_shape_across_processes - mismatched models fail loudly at construction."""
    _run(_w_shapes)


def _w_order(rank, world, port):
    _setup(rank, world, port)
    import torch.nn.functional as F
    from pytorch_imageclassification_distributed_amd.parallel import GradReducer
    m = _model(0)
    red = GradReducer(m, bucket_cap_mb=0.5, first_bucket_mb=0.1)
    x, y = torch.randn(4, 3, 16, 16), torch.randint(0, 4, (4,))
    F.cross_entropy(m(x), y).backward()
    if rank == 1:  # pretend this rank saw a different gradient-ready order
        red._ready_order = list(reversed(red._ready_order))
    red.finish()
    import torch.distributed as dist
    layouts = [None] * world
    dist.all_gather_object(layouts, [(s, e, list(i)) for s, e, i in red.buckets])
    assert layouts[0] == layouts[1]  # rank 0's observed order is the one every rank rebuilt with
    dist.barrier()
    dist.destroy_process_group()  # clean gloo teardown before exit (an exit with live gloo threads can abort)


def test_bucket_rebuild_uses_rank0_order():
    _run(_w_order)


def _w_overlap(rank, world, port):
    _setup(rank, world, port)
    import torch.distributed as dist
    import torch.nn.functional as F
    from pytorch_imageclassification_distributed_amd.parallel import GradReducer
    m = _model(0)
    red = GradReducer(m, bucket_cap_mb=0.5, first_bucket_mb=0.1)
    seen = []  # gradients already arrived when each bucket's collective was issued
    orig = red._launch

    def spy(b):
        seen.append(sum(red.got))
        orig(b)
    red._launch = spy
    x, y = torch.randn(4, 3, 16, 16), torch.randint(0, 4, (4,))
    for _ in range(2):  # first step records the ready order, second runs on the rebuilt buckets
        seen.clear()
        red.begin()
        F.cross_entropy(m(x), y).backward()
        nb, launched = len(red.buckets), sum(red.launched)
        assert nb > 2
        # every bucket's all-reduce is already issued when backward returns (nothing waits for finish())
        assert launched == nb, (launched, nb)
        # and the first one went out while most gradients were still being computed
        assert seen[0] < len(red.params) // 2, (seen[:3], len(red.params))
        red.finish()
    dist.barrier()
    dist.destroy_process_group()


def test_bucket_collectives_issued_during_backward():
    """the bucket all-reduces are in flight before backward ends (DDP-style overlap), not
    issued from finish()."""
    _run(_w_overlap)


def _w_syncbn_guard(rank, world, port):
    _setup(rank, world, port)
    import torch.distributed as dist
    import torch.nn as nn
    from pytorch_imageclassification_distributed_amd.parallel import SyncBNMismatchError, check_syncbn_consistency
    torch.manual_seed(0)
    m = nn.Sequential(nn.Conv2d(3, 8, 3), nn.BatchNorm2d(8), nn.ReLU(), nn.Conv2d(8, 8, 1), nn.BatchNorm2d(8))
    check_syncbn_consistency(m, None, "identical")  # same buffers on both ranks: passes
    if rank == 1:
        with torch.no_grad():
            m[4].running_var[3] += 1e-6  # one element on one rank
    with pytest.raises(SyncBNMismatchError, match="differ between ranks"):
        check_syncbn_consistency(m, None, "perturbed")
    dist.barrier()
    dist.destroy_process_group()


def test_syncbn_consistency_guard():
    """Steady-state SyncBN guard: diverged running statistics on any rank stop the run on
    every rank (the check is collective, so all ranks raise together)."""
    _run(_w_syncbn_guard)


# ---------------------------------------------------------------------------
def _bench(args, env_extra=None, timeout=300):
    import json
    import subprocess
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_PORT")}
    env.update(env_extra or {})
    r = subprocess.run([sys.executable, os.path.join(root, "bench.py")] + args, capture_output=True, text=True,
                       timeout=timeout, env=env, cwd=root)
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    return r.returncode, (json.loads(lines[-1]) if lines else None), r.stderr


def test_bench_gpus_flag_launches_the_ranks():
    """``bench.py --gpus 2`` with no launcher starts 2 ranks itself (torch.distributed.run, 127.0.0.1) and the
    JSON line reports the whole job: n_gpus 2, dp2, global batch = 2 x per-GPU batch (gloo CPU rehearsal)."""
    rc, out, err = _bench(["--gpus", "2", "--device", "cpu", "--model", "resnet18", "--image-size", "32",
                           "--batch", "4", "--steps", "2", "--warmup", "1"])
    assert rc == 0, err[-2000:]
    assert out["n_gpus"] == 2 and out["config"]["parallelism"] == "dp2" and out["config"]["global_batch"] == 8
    assert out["steps"] == 2 and out["value"] > 0 and "not a benchmark" in out["metric"]


def test_bench_eight_rank_rehearsal():
    """The driver's N = 8 launch shape, rehearsed on the CPU over gloo: ``bench.py --gpus 8`` starts 8 ranks,
    reports n_gpus 8 / dp8 / global batch 8 x per-GPU, the time of the slowest rank (its index and every
    rank's ms/step are in the line) and SyncBN on (reference semantics at N > 1); ``--data host`` is
    rehearsed as ``--data device`` (the host loader is GPU-only)."""
    rc, out, err = _bench(["--gpus", "8", "--device", "cpu", "--model", "resnet18", "--image-size", "32",
                           "--batch", "2", "--steps", "2", "--warmup", "1", "--data", "host"], timeout=600)
    assert rc == 0, err[-3000:]
    assert out["n_gpus"] == 8 and out["config"]["parallelism"] == "dp8" and out["config"]["global_batch"] == 16
    assert out["config"]["sync_bn"] is True and "not a benchmark" in out["metric"]
    ranks = out["rank_ms_per_step"]
    assert len(ranks) == 8 and 0 <= out["slowest_rank"] < 8
    assert ranks[out["slowest_rank"]] == max(ranks)
    assert abs(out["ms_per_step"] - max(ranks)) <= 0.01 * max(ranks) + 0.01  # the reported time is the max
    assert "rehearsing with --data device" in err


def test_scale_sweep_script_rehearsal(tmp_path):
    """scripts/scale_sweep.sh (the 8-GPU node's sweep: N x SyncBN x bucket MiB x transport dtype x gradient
    backend) runs end to end as a CPU rehearsal: 2 gloo ranks, one bucket size, both transport dtypes; one
    JSON line per run, tagged with its sweep point."""
    import json
    import subprocess
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    out = tmp_path / "sweep.jsonl"
    env = dict(os.environ, NS="2", SYNCBN="on", BUCKETS="8", COMMS="fp32 bf16", BACKENDS="pg", REF="0",
               BACKEND="gloo", BATCH="2", STEPS="1", WARMUP="1", MODEL="resnet18", IMAGE_SIZE="32",
               EXTRA="--device cpu", OUT=str(out), TIMEOUT="600", GRAFT_REPO_ROOT=root)
    r = subprocess.run(["bash", os.path.join(root, "scripts", "scale_sweep.sh")], env=env, capture_output=True,
                       text=True, timeout=900)
    assert r.returncode == 0, (r.stdout[-2000:], r.stderr[-2000:])
    rows = [json.loads(line) for line in out.read_text().splitlines()]
    assert [row["tag"] for row in rows] == ["resnet18_n2_sbon_b8_fp32_pg", "resnet18_n2_sbon_b8_bf16_pg"]
    for row in rows:
        run = row["run"]
        assert run["n_gpus"] == 2 and run["config"]["sync_bn"] is True and run["value"] > 0


def test_bench_refuses_a_world_size_mismatch():
    """A single rank asked for ``--gpus 2`` under a launcher-provided WORLD_SIZE=1 exits non-zero without a
    (mislabelled) JSON line."""
    rc, out, _ = _bench(["--gpus", "2", "--device", "cpu", "--model", "resnet18", "--image-size", "32",
                         "--batch", "2", "--steps", "1", "--warmup", "1"],
                        env_extra={"WORLD_SIZE": "1", "RANK": "0", "LOCAL_RANK": "0", "MASTER_ADDR": "127.0.0.1",
                                   "MASTER_PORT": str(_port())})
    assert rc == 2 and out is None


# ---------------------------------------------------------------------------
def _w_resume(rank, world, port, ck, port2):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank),
                      WORLD_SIZE=str(world), LOCAL_RANK=str(rank))
    import train
    from pytorch_imageclassification_distributed_amd.utils import load_checkpoint
    args = ["--synthetic", "--model", "resnet18", "--image-size", "32", "--device", "cpu", "--batchsize", "8",
            "--num-workers", "0", "--synthetic-train-size", "64", "--synthetic-val-size", "16", "--no-progress",
            "--val-batchsize", "8", "--steps-per-epoch", "2", "--val-steps", "1", "--latest-every", "1",
            "--ckpt-dir", ck]
    train.main(args + ["--epochs", "1", "--resume", "none"])
    import time
    path = os.path.join(ck, "resnet18", "latest_model")
    for _ in range(600):  # rank 0 writes it (temp file + rename): wait until it exists
        if os.path.exists(path):
            break
        time.sleep(0.1)
    lt = load_checkpoint(path)
    assert len(lt["rng_ranks"]) == world
    # the ranks' streams differ (per-rank seeding), and each entry is that rank's own
    assert not torch.equal(lt["rng_ranks"][0]["torch"], lt["rng_ranks"][1]["torch"])
    assert torch.equal(lt["rng"]["torch"], lt["rng_ranks"][0]["torch"])
    mine = lt["rng_ranks"][rank]["torch"]
    from pytorch_imageclassification_distributed_amd.engine import trainer as tm
    seen = {}
    orig = tm.Trainer.maybe_resume

    def spy(self):
        orig(self)
        seen["how"] = getattr(self, "rng_restored", None)
        seen["state"] = torch.get_rng_state().clone()
    tm.Trainer.maybe_resume = spy
    os.environ["MASTER_PORT"] = str(port2)  # a fresh rendezvous for the second process group
    try:
        hist = train.main(args + ["--epochs", "2", "--resume", "latest"])
    finally:
        tm.Trainer.maybe_resume = orig
    assert [h["epoch"] for h in hist] == [1]
    assert seen["how"] == "rank" and torch.equal(seen["state"], mine)


def test_resume_restores_each_ranks_rng(tmp_path):
    """2-rank gloo: latest_model stores every rank's random streams (rng_ranks), and --resume latest gives
    each rank back its own - not rank 0's (reference train.py:183-188 saves from rank 0 only)."""
    port, port2 = _port(), _port()
    mp.spawn(_w_resume, args=(2, port, str(tmp_path), port2), nprocs=2, join=True)


# ---------------------------------------------------------------------------
class _Probe:
    def __init__(self, done=False):
        self.done = done

    def query(self):
        return self.done


def test_comm_watchdog_aborts_on_async_error():
    """The native communicator's watchdog (parallel/rccl.py CommWatchdog): an asynchronous RCCL error aborts
    the communicator and ends the process (os._exit by default; a recorder here)."""
    import time

    from pytorch_imageclassification_distributed_amd.parallel.rccl import CommWatchdog
    err, calls = [0], []
    wd = CommWatchdog(lambda: err[0], lambda: calls.append("abort"), timeout=60, interval=0.01,
                      on_fatal=lambda m: calls.append(m))
    wd.arm(_Probe(True))
    time.sleep(0.1)
    assert calls == [] and wd.fired is None
    err[0] = 6  # ncclRemoteError
    for _ in range(200):
        if len(calls) == 2:
            break
        time.sleep(0.01)
    assert calls[0] == "abort" and "asynchronous error 6" in calls[1]
    wd.stop()


def test_comm_watchdog_ends_a_hung_collective():
    """Collectives whose completion event never fires within the deadline abort the communicator and end the
    process - a dead peer cannot leave a rank waiting forever (the PG timeout does not watch this comm)."""
    import subprocess
    import sys
    code = ("import time\n"
            "from pytorch_imageclassification_distributed_amd.parallel.rccl import CommWatchdog\n"
            "class P:\n    def query(self): return False\n"
            "wd = CommWatchdog(lambda: 0, lambda: print('aborted', flush=True), timeout=0.3, interval=0.05)\n"
            "wd.arm(P())\n"
            "time.sleep(30)\n"
            "print('not reached', flush=True)\n")
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    r = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True, timeout=60, cwd=root)
    assert r.returncode == 13, (r.returncode, r.stdout, r.stderr)
    assert "aborted" in r.stdout and "not reached" not in r.stdout and "have not completed" in r.stderr


def test_close_all_stops_watchdogs_before_teardown():
    """parallel.dist.destroy() -> rccl.close_all() stops every live watchdog before any communicator closes, so a
    poll that sees the closed communicator (formerly -1 from the native side) never ends a clean run non-zero."""
    import time

    from pytorch_imageclassification_distributed_amd.parallel import rccl as R
    err, calls = [0], []
    wd = R.CommWatchdog(lambda: err[0], lambda: calls.append("abort"), timeout=60, interval=0.01,
                        on_fatal=lambda m: calls.append(m))
    assert wd in R._WATCHDOGS
    R.close_all()
    assert wd not in R._WATCHDOGS and not wd._t.is_alive()
    err[0] = -1
    time.sleep(0.1)
    assert calls == [] and wd.fired is None


def test_grad_reducer_wires_the_watchdog(monkeypatch):
    """GradReducer(comm='rccl') arms the watchdog with one completion event per step and check() raises on
    an async error (a stub communicator stands in for RcclComm: RCCL needs GPUs)."""
    import types

    from pytorch_imageclassification_distributed_amd.parallel import rccl as R
    from pytorch_imageclassification_distributed_amd.parallel.reducer import GradReducer

    class FakeComm:
        def __init__(self, group=None, device=None):
            self.err = 0
            self.closed = None

        def async_error(self):
            return self.err

        def check(self):
            if self.err:
                raise RuntimeError(f"RCCL communicator error {self.err}")

        def close(self, abort=False):
            self.closed = abort

    monkeypatch.setattr(R, "RcclComm", FakeComm)
    m = torch.nn.Linear(4, 2)
    red = GradReducer(m, comm="rccl", force_collectives=True, broadcast=False)
    assert isinstance(red.watchdog, R.CommWatchdog) and red.watchdog.timeout == 600.0
    red.check()
    red.rccl.err = 2
    with pytest.raises(RuntimeError, match="error 2"):
        red.check()
    red.rccl.err = 0
    comm = red.rccl
    red.close()
    assert red.watchdog is None and red.rccl is None and comm.closed is False


# ---------------------------------------------------------------------------
def _w_syncbn_guard(rank, world, port):
    _setup(rank, world, port)
    from pytorch_imageclassification_distributed_amd.parallel.peer import SyncBNMismatchError, check_syncbn_consistency
    m = torch.nn.Sequential(torch.nn.BatchNorm2d(4), torch.nn.BatchNorm2d(3))
    check_syncbn_consistency(m)  # equal on both ranks
    if rank == 1:
        m[1].running_mean[2] += 1e-6
    with pytest.raises(SyncBNMismatchError, match="differ between ranks"):
        check_syncbn_consistency(m)
    if rank == 1:
        m[1].running_mean[2] -= 1e-6
        m[0].running_var[1] = float("nan")
    with pytest.raises(SyncBNMismatchError, match="some ranks only.*transport fault"):
        check_syncbn_consistency(m)  # one rank non-finite: the statistics differ (a stale / torn slot)
    m[0].running_var[1] = float("nan")
    with pytest.raises(SyncBNMismatchError, match="every rank.*diverged"):
        check_syncbn_consistency(m)  # every rank non-finite: divergence


def test_syncbn_guard_flat_checksum_and_nonfinite():
    """The SyncBN guard (one flat checksum + one all-reduce): a one-ulp difference on one rank is a mismatch;
    a NaN running statistic on every rank is divergence; on one rank only, a transport mismatch."""
    _run(_w_syncbn_guard)


def test_syncbn_guard_runs_on_its_own_interval(monkeypatch, tmp_path):
    """The guard (a collective + host sync) runs every --syncbn-check-every steps and at epoch end, not at
    every log interval (--log-interval defaults to 1)."""
    import train
    from pytorch_imageclassification_distributed_amd.engine import trainer as tm
    calls = []
    monkeypatch.setattr(tm, "check_syncbn_consistency", lambda *a, **k: calls.append("sum"))
    monkeypatch.setattr(tm, "check_peer_errors", lambda *a, **k: calls.append("err"))
    orig = tm.Trainer._build_model

    def build(self):
        orig(self)
        self.syncbn_peer = True  # pretend the peer transport is up (CPU: it never is)
    monkeypatch.setattr(tm.Trainer, "_build_model", build)
    args = ["--synthetic", "--model", "resnet18", "--image-size", "32", "--device", "cpu", "--batchsize", "8",
            "--num-workers", "0", "--synthetic-train-size", "48", "--synthetic-val-size", "8", "--no-progress",
            "--epochs", "1", "--resume", "none", "--ckpt-dir", str(tmp_path)]
    train.main(args + ["--syncbn-check-every", "2"])  # 6 steps: after steps 2, 4, 6 and at epoch end
    assert calls.count("sum") == 4
    calls.clear()
    train.main(args)  # default interval 100: epoch end only
    assert calls.count("sum") == 1
