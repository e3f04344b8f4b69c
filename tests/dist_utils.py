"""Multi-process test harness: spawn `world` CPU ranks on gloo (127.0.0.1), run `fn(rank, world, *args)`
and collect each rank's return value (pickled through a queue)."""
import os
import socket
import sys
import traceback

import torch.multiprocessing as mp

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _free_port():
    """A free port BELOW the kernel's ephemeral range (32768+): an ephemeral port released here can
    be handed to another socket's outgoing connection before rank 0 binds it (EADDRINUSE)."""
    import random
    for _ in range(100):
        p = random.randrange(20000, 32000)
        s = socket.socket()
        try:
            s.bind(("127.0.0.1", p))
            return p
        except OSError:
            continue
        finally:
            s.close()
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, fn, args, q):
    try:
        if ROOT not in sys.path:
            sys.path.insert(0, ROOT)
        os.environ.update(RANK=str(rank), WORLD_SIZE=str(world), LOCAL_RANK=str(rank), MASTER_ADDR="127.0.0.1",
                          MASTER_PORT=str(port))
        import torch
        torch.set_num_threads(1)
        from shuffle_exchange_amd import comm
        comm.init_distributed(dist_backend="gloo", verbose=False)
        out = fn(rank, world, *args)
        import io
        buf = io.BytesIO()
        torch.save(out, buf)  # plain bytes: no shared-memory fds outliving the child
        q.put((rank, "ok", buf.getvalue()))
        import torch.distributed as td
        td.barrier()
        td.destroy_process_group()
        from shuffle_exchange_amd.parallel import groups
        groups.reset()
    except Exception:
        q.put((rank, "err", traceback.format_exc()))


def run_dist(fn, world, *args, timeout=240):
    for attempt in range(3):  # a rendezvous port taken between probe and bind: new port, same run
        try:
            return _run_dist(fn, world, *args, timeout=timeout)
        except RuntimeError as e:
            if "EADDRINUSE" not in str(e) or attempt == 2:
                raise


def _run_dist(fn, world, *args, timeout=240):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, fn, args, q)) for r in range(world)]
    for p in procs:
        p.start()
    results = {}
    try:
        for _ in range(world):
            rank, status, out = q.get(timeout=timeout)
            if status == "err":
                raise RuntimeError(f"rank {rank} failed:\n{out}")
            import io
            import torch
            results[rank] = torch.load(io.BytesIO(out), weights_only=True)
    finally:
        for p in procs:
            p.join(timeout=30)
            if p.is_alive():
                p.kill()
    return [results[r] for r in range(world)]
