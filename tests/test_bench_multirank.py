"""bench.py's N > 1 control flow (C4) on CPU: two ranks launched like the
driver's torch.distributed.run, with the renderer replaced by a recording fake
whose barrier / max-over-ranks / all-reduce run over gloo. Checks that the
driver's command line (--steps 20 --warmup 5, fewer passes than the composite
interval) still ends the timed region with a radiance all-reduce (its host
readback follows the region), that ranks use distinct seed streams, that the rendezvous
hands every rank the same unique id, and that rank 0 prints one JSON line with
the whole-job value."""
import json
import os
import socket
import subprocess
import sys
import textwrap

import pytest
from pathlib import Path

REPO = Path(__file__).resolve().parents[1]

DRIVER = textwrap.dedent('''
    import importlib.util, json, os, sys, time
    sys.argv = ["bench.py"] + json.loads(os.environ["BENCH_ARGV"])
    spec = importlib.util.spec_from_file_location("bench", os.environ["BENCH_PATH"])
    bench = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(bench)
    import numpy as np
    import torch.distributed as dist

    LOG = []

    class Fake:
        def __init__(self, R, device=0, layout=1, devices=None, transport=0):
            if devices is not None:
                ndev = int(os.environ.get("FAKE_NDEV", "8"))
                bad = [d for d in devices if d >= ndev]
                if bad:  # the library refuses an ordinal past the device count
                    raise bench.vptmcm.VptError(-1, f"devices: {bad[0]} is not a device ordinal ({ndev} devices)")
                LOG.append(["create_group", R, list(devices), transport, layout])
            else:
                LOG.append(["create", R, device, layout])
            self.t0, self.launches = None, 0
        def set_volume(self, v): LOG.append(["volume", list(v.shape)])
        def set_material_tf(self, tf): pass
        def set_light(self, spd, d): pass
        def set_spectrum(self, s): pass
        def set_params(self, **kw): pass
        def comm_init(self, uid, world, rank):
            LOG.append(["comm_init", bytes(uid).hex()[:16], world, rank])
            if os.environ.get("FAKE_HANG_INIT") == os.environ["RANK"]:
                time.sleep(3600)  # this rank's communicator init never returns
            os.write(1, ("RCCL version : (banner on fd 1, as RCCL writes it)" + chr(10)).encode())
            dist.init_process_group("gloo", rank=rank, world_size=world,
                                    timeout=__import__("datetime").timedelta(seconds=60))
        def barrier(self): dist.barrier()
        def reset(self, mvp, seed): LOG.append(["reset", int(seed)])
        def render_passes(self, mvp, seeds):
            LOG.append(["passes", [int(s) for s in seeds]])
            self.launches += 1
            time.sleep(float(os.environ.get("FAKE_PASS_SLEEP", "0")))
        def synchronize(self): pass
        def enable_kernel_timing(self, on):
            self.t0, self.launches = time.perf_counter(), 0
            LOG.append(["timing"] if on else ["timing_off"])
        def kernel_time(self):
            return (time.perf_counter() - self.t0) * 1e3 + 1e-3, self.launches
        def last_launch(self):
            return {"mode": 2, "tpl": 5, "spec": True, "macro": False, "passes": 32, "launches": 0}
        def allreduce_radiance(self, inline=False, sharded=False):
            LOG.append(["allreduce_inline" if inline else "allreduce", bool(sharded)])
            if os.environ.get("FAKE_DIE_RANK") == os.environ["RANK"]:
                os._exit(3)  # this rank dies before its first composite
        def read_composite(self):
            LOG.append(["composite"])
            return np.zeros((4, 4, 3), np.float32), np.zeros((4, 4), np.float32)
        def composite(self):
            LOG.append(["group_composite"])
        def read_composite_all(self):
            LOG.append(["read_group_composite"])
        def allreduce_host(self, vals, op="sum"):
            t = __import__("torch").tensor(np.asarray(vals, np.float64))
            dist.all_reduce(t, op=dist.ReduceOp.MAX if op == "max" else dist.ReduceOp.SUM)
            return t.numpy()
        def close(self):
            if dist.is_initialized():
                dist.destroy_process_group()

    bench.vptmcm.Renderer = Fake
    bench.vptmcm.unique_id = lambda: os.urandom(128)
    bench.entry()
    Path = __import__("pathlib").Path
    Path(os.environ["LOG_OUT"]).write_text(json.dumps(LOG))
''')


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


@pytest.mark.parametrize("world", [2, 4])
def test_bench_two_ranks_driver_command_line(tmp_path, world):
    port = _free_port()
    argv = ["--gpus", str(world), "--steps", "20", "--warmup", "5", "--volume", "16",
            "--resolution", "16", "--cpu-seconds", "0"]
    procs = []
    for rank in range(world):
        env = dict(os.environ, RANK=str(rank), LOCAL_RANK=str(rank), WORLD_SIZE=str(world),
                   MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), BENCH_ARGV=json.dumps(argv),
                   BENCH_PATH=str(REPO / "bench.py"), LOG_OUT=str(tmp_path / f"log{rank}.json"),
                   TORCHELASTIC_RUN_ID=f"t{port}")
        procs.append(subprocess.Popen([sys.executable, "-c", DRIVER], env=env, stdout=subprocess.PIPE,
                                      stderr=subprocess.PIPE, text=True, cwd=str(tmp_path)))
    outs = [p.communicate(timeout=300) for p in procs]
    for p, (o, e) in zip(procs, outs):
        assert p.returncode == 0, o + e
    line = [ln for ln in outs[0][0].splitlines() if ln.startswith("{")]
    assert len(line) == 1 and not [ln for o in outs[1:] for ln in o[0].splitlines() if ln.startswith("{")]
    # stdout carries rank 0's JSON line and nothing else (RCCL's banner goes to stderr)
    assert [ln for ln in outs[0][0].splitlines() if ln.strip()] == line
    assert all(not o[0].strip() for o in outs[1:])
    assert all("RCCL version" in o[1] for o in outs)
    rec = json.loads(line[0])
    assert rec["n_gpus"] == world and rec["steps"] == 20 and rec["warmup"] == 5
    assert rec["value"] > 0 and rec["config"]["workload"].startswith("custom: 16^3")
    assert rec["per_pass_allreduce"]["steps"] == 64 and rec["per_pass_allreduce"]["value"] > 0
    logs = [json.loads((tmp_path / f"log{r}.json").read_text()) for r in range(world)]
    uids = {e[1] for lg in logs for e in lg if e[0] == "comm_init"}
    assert len(uids) == 1, "ranks must share rank 0's unique id"
    for r, lg in enumerate(logs):
        assert ["create", 16, r, 3] in lg  # one GPU per local rank (COLUMN4, the default layout)
        t = [e[0] for e in lg].index("timing")
        after = lg[t + 1:]
        c1 = [e[0] for e in after].index("composite")
        timed, rest = after[:c1 + 1], after[c1 + 1:]  # the main region, then the per-pass one
        kinds = [e[0] for e in timed]
        assert sum(len(e[1]) for e in timed if e[0] == "passes") == 20
        last_pass = max(i for i, k in enumerate(kinds) if k == "passes")
        # the region ends with a composite, the last one inline (about to be read)
        assert kinds[last_pass + 1] == "allreduce_inline", "timed region must end with a composite"
        assert kinds.index("composite") > last_pass
        # per-pass compositing region: 64 one-pass launches, each followed by an all-reduce
        rk = [e[0] for e in rest if e[0] in ("passes", "allreduce", "allreduce_inline")]
        assert rk[:128] == ["passes", "allreduce"] * 63 + ["passes", "allreduce_inline"]
        assert all(len(e[1]) == 1 for e in rest if e[0] == "passes")
        # the composites reduce-scatter by default (--shard-composite on)
        assert all(e[1] for e in lg if e[0] in ("allreduce", "allreduce_inline"))
    seeds = [[s for e in lg if e[0] == "passes" for s in e[1]] for lg in logs]
    for a in range(world):
        for b in range(a + 1, world):
            assert not set(seeds[a]) & set(seeds[b]), "ranks must use distinct seed streams"


def test_bench_rank_death_ends_the_job(tmp_path):
    """A rank that dies before the first radiance all-reduce must not leave the
    others hanging: rank 0's next collective fails and bench.py exits non-zero
    within the timeout, printing no result line. (On the GPU the library's RCCL
    watchdog does the same: vptmcm_comm_* poll ncclCommGetAsyncError and abort
    after VPTMCM_COMM_TIMEOUT_MS.)"""
    import time
    port = _free_port()
    argv = ["--gpus", "2", "--steps", "20", "--warmup", "5", "--volume", "16",
            "--resolution", "16", "--cpu-seconds", "0"]
    procs = []
    t0 = time.monotonic()
    for rank in range(2):
        env = dict(os.environ, RANK=str(rank), LOCAL_RANK=str(rank), WORLD_SIZE="2",
                   MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), BENCH_ARGV=json.dumps(argv),
                   BENCH_PATH=str(REPO / "bench.py"), LOG_OUT=str(tmp_path / f"log{rank}.json"),
                   TORCHELASTIC_RUN_ID=f"d{port}", FAKE_DIE_RANK="1")
        procs.append(subprocess.Popen([sys.executable, "-c", DRIVER], env=env, stdout=subprocess.PIPE,
                                      stderr=subprocess.PIPE, text=True, cwd=str(tmp_path)))
    outs = [p.communicate(timeout=240) for p in procs]
    took = time.monotonic() - t0
    assert procs[1].returncode == 3
    assert procs[0].returncode != 0, outs[0]
    assert not [ln for ln in outs[0][0].splitlines() if ln.startswith("{")]
    assert took < 200, took


def test_bench_missing_rank_fails_in_the_rendezvous(tmp_path):
    """World 2 where rank 1 never starts: rank 0 must fail in the all-ranks-present
    rendezvous with ECOMM before any communicator call (no comm_init is made, so
    no RCCL bootstrap is left waiting for the missing peer), within the bound."""
    import time
    port = _free_port()
    argv = ["--gpus", "2", "--steps", "20", "--warmup", "5", "--volume", "16",
            "--resolution", "16", "--cpu-seconds", "0"]
    env = dict(os.environ, RANK="0", LOCAL_RANK="0", WORLD_SIZE="2",
               MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), BENCH_ARGV=json.dumps(argv),
               BENCH_PATH=str(REPO / "bench.py"), LOG_OUT=str(tmp_path / "log0.json"),
               TORCHELASTIC_RUN_ID=f"m{port}", VPTMCM_COMM_TIMEOUT_MS="1500")
    t0 = time.monotonic()
    p = subprocess.run([sys.executable, "-c", DRIVER], env=env, capture_output=True, text=True,
                       cwd=str(tmp_path), timeout=120)
    took = time.monotonic() - t0
    assert p.returncode == 3, p.stdout + p.stderr
    assert "vptmcm error -5" in p.stderr and "never joined" in p.stderr and "[1]" in p.stderr
    assert "RCCL version" not in p.stderr  # the fake comm_init (and its banner) never ran
    assert not [ln for ln in p.stdout.splitlines() if ln.startswith("{")]
    assert took < 60, took


def test_bench_hung_comm_init_ends_every_rank(tmp_path):
    """Both ranks pass the rendezvous, then rank 1's communicator init never
    returns (a peer that dies inside RCCL's bootstrap): rank 0's init waits for
    it and cannot be bounded from inside RCCL, so bench.py's init watchdog ends
    each process with exit 3 after VPTMCM_COMM_TIMEOUT_MS."""
    import time
    port = _free_port()
    argv = ["--gpus", "2", "--steps", "20", "--warmup", "5", "--volume", "16",
            "--resolution", "16", "--cpu-seconds", "0"]
    procs = []
    t0 = time.monotonic()
    for rank in range(2):
        env = dict(os.environ, RANK=str(rank), LOCAL_RANK=str(rank), WORLD_SIZE="2",
                   MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), BENCH_ARGV=json.dumps(argv),
                   BENCH_PATH=str(REPO / "bench.py"), LOG_OUT=str(tmp_path / f"log{rank}.json"),
                   TORCHELASTIC_RUN_ID=f"h{port}", FAKE_HANG_INIT="1", VPTMCM_COMM_TIMEOUT_MS="4000")
        procs.append(subprocess.Popen([sys.executable, "-c", DRIVER], env=env, stdout=subprocess.PIPE,
                                      stderr=subprocess.PIPE, text=True, cwd=str(tmp_path)))
    outs = [p.communicate(timeout=120) for p in procs]
    took = time.monotonic() - t0
    for p, (o, e) in zip(procs, outs):
        assert p.returncode == 3, o + e
        assert "did not return within 4 s" in e
        assert not [ln for ln in o.splitlines() if ln.startswith("{")]
    assert took < 90, took


def _run_launcherless(tmp_path, argv, **env_extra):
    env = {k: v for k, v in os.environ.items()
           if k not in ("RANK", "LOCAL_RANK", "WORLD_SIZE", "MASTER_ADDR", "MASTER_PORT")}
    env.update(BENCH_ARGV=json.dumps(argv), BENCH_PATH=str(REPO / "bench.py"),
               LOG_OUT=str(tmp_path / "log.json"), **env_extra)
    return subprocess.run([sys.executable, "-c", DRIVER], env=env, capture_output=True, text=True,
                          cwd=str(tmp_path), timeout=300)


@pytest.mark.parametrize("transport", ["peer", "rccl"])
def test_bench_gpus4_without_launcher_is_one_device_list_handle(tmp_path, transport):
    """`python bench.py --gpus 4` with no launcher: one
    process, ONE 4-device handle over devices 0..3 (the north_star's JS host
    shape), the timed region ends with the device-list composite, the line
    reports n_gpus 4, the parallelism and the composite transport, and the
    whole-job value counts all four replicas' photon-steps."""
    argv = ["--gpus", "4", "--steps", "20", "--warmup", "5", "--volume", "16", "--resolution", "16",
            "--cpu-seconds", "0", "--transport", transport]
    p = _run_launcherless(tmp_path, argv, FAKE_NDEV="4", FAKE_PASS_SLEEP="0.002")
    assert p.returncode == 0, p.stdout + p.stderr
    lines = [ln for ln in p.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1
    rec = json.loads(lines[0])
    assert rec["n_gpus"] == 4 and rec["config"]["workload"].startswith("custom: 16^3")
    assert rec["config"]["devices"] == [0, 1, 2, 3]
    assert rec["config"]["composite_transport"] == {"peer": "peer-sharded", "rccl": "rccl-reduce"}[transport]
    assert "one process" in rec["config"]["parallelism"] and "x4" in rec["config"]["parallelism"]
    assert rec["cpu_baseline"] is None and rec["unfused"] is None
    log = json.loads((tmp_path / "log.json").read_text())
    creates = [e for e in log if e[0].startswith("create")]
    assert creates == [["create_group", 16, [0, 1, 2, 3], 0 if transport == "peer" else 1, 3]]
    assert not [e for e in log if e[0] in ("comm_init", "allreduce", "allreduce_inline")]
    t = [e[0] for e in log].index("timing")
    after = [e[0] for e in log[t + 1:]]
    last_pass = max(i for i, k in enumerate(after[:after.index("read_group_composite")]) if k == "passes")
    assert "group_composite" in after[last_pass:after.index("read_group_composite")], \
        "timed region must end with the composite"
    # the whole job: 4 replicas x R^2 x S x steps over the region's wall time
    assert abs(rec["value"] - 4 * 16 * 16 * 8 * 20 / (rec["roofline"]["region_wall_us"] * 1e-6) / 1e6) \
        <= 0.01 * rec["value"]


def test_bench_gpus2_with_one_visible_device_fails(tmp_path):
    """Fewer visible devices than --gpus and no launcher: exit non-zero with the
    library's reason, no result line (never a silent one-GPU run)."""
    argv = ["--gpus", "2", "--steps", "20", "--warmup", "5", "--volume", "16", "--resolution", "16",
            "--cpu-seconds", "0"]
    p = _run_launcherless(tmp_path, argv, FAKE_NDEV="1")
    assert p.returncode != 0
    assert "not a device ordinal" in p.stderr and "device-list handle" in p.stderr
    assert not [ln for ln in p.stdout.splitlines() if ln.startswith("{")]


def test_bench_devices_override_repeats_a_device(tmp_path):
    """VPTMCM_BENCH_DEVICES (test-only) repeats device 0: the control flow of
    --gpus 2 on a one-GPU box."""
    argv = ["--gpus", "2", "--steps", "20", "--warmup", "5", "--volume", "16", "--resolution", "16",
            "--cpu-seconds", "0"]
    p = _run_launcherless(tmp_path, argv, FAKE_NDEV="1", VPTMCM_BENCH_DEVICES="0,0")
    assert p.returncode == 0, p.stdout + p.stderr
    rec = json.loads([ln for ln in p.stdout.splitlines() if ln.startswith("{")][0])
    assert rec["n_gpus"] == 2 and rec["config"]["devices"] == [0, 0]
