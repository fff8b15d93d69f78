"""The RCCL watchdog under repetition: a 2-rank communicator whose second rank
never joins, four times in one process (VPTMCM_COMM_TRACE=1 for the stages).
Each attempt must fail with ECOMM after VPTMCM_COMM_TIMEOUT_MS (3 s) plus at
most the bounded abort (2 s)."""
import os, sys, time
sys.path[:0] = ["vpt-spectral-volume-rendering_amd/python"]
import vptmcm
from vptmcm import configs as cf
os.environ["VPTMCM_COMM_TIMEOUT_MS"] = "3000"
for k in range(4):
    g = vptmcm.Renderer(32, device=0)
    t0 = time.monotonic()
    try:
        g.comm_init(vptmcm.unique_id(), 2, 0)
        print("unexpected success")
    except vptmcm.VptError as e:
        print(f"run {k}: {time.monotonic() - t0:.2f} s: {e}", flush=True)
    g.close()
