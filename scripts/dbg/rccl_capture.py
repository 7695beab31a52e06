"""Can RCCL (ProcessGroupNCCL) collectives be captured into a hipGraph on this stack?  One
collective per process (a failure can abort the process), world 1 on the box's GPU:

    python scripts/dbg/rccl_capture.py            # runs every case in its own child process
    python scripts/dbg/rccl_capture.py CASE       # one case
Prints one JSON line per case: captured, replayed, result correct, error."""
import json
import os
import subprocess
import sys

# the cases that crash the capturing process on this stack (r6s5 / r6s6) come last: the run stops at
# the first crash
CASES = ["all_reduce", "all_reduce_async", "all_gather_async", "reduce_scatter_async", "rs_ag_chain",
         "rs_ag_side_chain", "all_to_all_async", "side_stream_chain"]


def run_case(case: str) -> dict:
    import torch
    import torch.distributed as dist

    os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
    dist.init_process_group("nccl", rank=0, world_size=1, device_id=torch.device("cuda", 0))
    dev = torch.device("cuda", 0)
    x = torch.arange(1024, device=dev, dtype=torch.float32)
    out = torch.empty_like(x)
    dist.all_reduce(x.clone())  # communicator up before the capture
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    rec = {"case": case, "captured": False, "replayed": False, "correct": None, "error": None}
    side = torch.cuda.Stream()
    try:
        s = torch.cuda.Stream()
        s.wait_stream(torch.cuda.current_stream())
        with torch.cuda.graph(g):
            y = x * 2
            if case == "all_reduce":
                dist.all_reduce(y)
            elif case == "all_reduce_async":
                dist.all_reduce(y, async_op=True).wait()
            elif case == "all_to_all_async":
                dist.all_to_all_single(out, y, async_op=True).wait()
                y = out
            elif case == "all_gather_async":
                dist.all_gather_into_tensor(out, y, async_op=True).wait()
                y = out
            elif case == "reduce_scatter_async":
                dist.reduce_scatter_tensor(out, y, async_op=True).wait()
                y = out
            elif case == "rs_ag_chain":  # the bucketer's capture path: all on the capturing stream
                dist.reduce_scatter_tensor(out, y, async_op=True).wait()
                z = out + 1
                dist.all_gather_into_tensor(out, z, async_op=True).wait()
                y = out
            elif case == "rs_ag_side_chain":  # fp32 reduce-scatter, cast on a side stream, all-gather
                w1 = dist.reduce_scatter_tensor(out, y, async_op=True)
                with torch.cuda.stream(side):
                    w1.wait()
                    z = out + 1
                    w2 = dist.all_gather_into_tensor(out, z, async_op=True)
                w2.wait()
                torch.cuda.current_stream().wait_stream(side)
                y = out
            elif case == "side_stream_chain":  # the bucketer's fp32_accum shape
                w1 = dist.all_to_all_single(out, y, async_op=True)
                with torch.cuda.stream(side):
                    w1.wait()
                    z = out + 1
                    w2 = dist.all_gather_into_tensor(out, z, async_op=True)
                w2.wait()
                torch.cuda.current_stream().wait_stream(side)
                y = out
            res = y + 0
        rec["captured"] = True
        g.replay()
        torch.cuda.synchronize()
        rec["replayed"] = True
        want = x * 2 + (1 if case in ("side_stream_chain", "rs_ag_side_chain", "rs_ag_chain") else 0)
        rec["correct"] = bool(torch.equal(res, want))
    except Exception as e:  # noqa: BLE001
        rec["error"] = f"{type(e).__name__}: {e}"[:300]
    print(json.dumps(rec), flush=True)
    os._exit(0)  # skip the watchdog / destroy path


def main() -> None:
    if len(sys.argv) > 1:
        run_case(sys.argv[1])
        return
    port = 29611
    for case in CASES:
        env = dict(os.environ, MASTER_PORT=str(port), MASTER_ADDR="127.0.0.1")
        port += 1
        r = subprocess.run([sys.executable, __file__, case], capture_output=True, text=True, timeout=120, env=env)
        line = [l for l in r.stdout.splitlines() if l.startswith("{")]
        if line:
            print(line[-1], flush=True)
        else:
            print(json.dumps({"case": case, "rc": r.returncode, "stderr": r.stderr[-600:]}), flush=True)
        if r.returncode < 0:  # a crashed child: nothing more runs on the GPU in this call
            break


if __name__ == "__main__":
    main()
