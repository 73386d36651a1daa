"""Probe hipIpc export/open of device allocations of different sizes / init states between two
processes on GPU 0 (each variant bounded by a deadline).  Parent never touches the GPU."""
import multiprocessing as mp
import sys
import time


def exporter(q_out, q_in, nbytes, init):
    import torch
    sys.path.insert(0, ".")
    from mxserve import ops
    torch.cuda.set_device(0)
    pre = torch.zeros(1 << 20, dtype=torch.uint8, device="cuda:0") if init == "second" else None
    t = (torch.zeros if init != "empty" else torch.empty)(nbytes, dtype=torch.uint8, device="cuda:0")
    torch.cuda.synchronize()
    h, off = ops.ext().ipc_export_pool(t)
    q_out.put((h, off))
    q_in.get(timeout=120)


def importer(q_out, q_in, delay):
    import torch
    sys.path.insert(0, ".")
    from mxserve import ops
    torch.cuda.set_device(0)
    h, off = q_in.get(timeout=60)
    time.sleep(delay)
    t0 = time.time()
    ops.ext().ipc_open_pool(h, off)
    q_out.put(time.time() - t0)


def main():
    ctx = mp.get_context("spawn")
    delay = float(sys.argv[1]) if len(sys.argv) > 1 else 0.0
    for gb, init in [(1, "zeros"), (4.5, "zeros"), (3, "zeros"), (1, "zeros"), (4.5, "zeros"), (2, "zeros"), (1.5, "zeros"), (0.5, "zeros")]:
        eo, ei, io, ii = ctx.Queue(), ctx.Queue(), ctx.Queue(), ctx.Queue()
        e = ctx.Process(target=exporter, args=(eo, ei, int(gb * (1 << 30)), init))
        i = ctx.Process(target=importer, args=(io, ii, delay))
        e.start()
        i.start()
        try:
            ii.put(eo.get(timeout=60))
            dt = io.get(timeout=20 + delay)
            print(f"{gb} GiB {init}: open {dt:.3f}s", flush=True)
        except Exception as ex:  # noqa: BLE001
            print(f"{gb} GiB {init}: FAILED/timeout ({type(ex).__name__})", flush=True)
        ei.put(1)
        for p in (e, i):
            p.join(timeout=10)
            if p.is_alive():
                p.kill()
                p.join()


if __name__ == "__main__":
    main()
