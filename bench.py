"""bench.py -- FEC encode+decode throughput of the MI355X engine (device-resident).

Workload per GPU (BASELINE.json configs[1] + configs[2]): 2^20 independent FEC blocks of
k = 16 source symbols x 1200 B; one step = RLC encode of r = 4 repairs for every block,
then RLC decode of every block with 4 random source erasures (all 4 repairs received),
recovered in place.  Inputs are synthetic (SplitMix64 bytes) and resident in HBM before the
timed region.  value = source payload (k * L * blocks, all ranks) / step time, in GiB/s:
each payload byte is both encoded and decoded inside one step.

Multi-GPU (torchrun, one process per GPU): blocks are partitioned, each rank owns its own
2^20 blocks (fbn offset by rank), there is no data-path collective (a FEC block never spans
GPUs); barrier + max-over-ranks timing only.  scaling = weak.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

HBM_PEAK_GBS = 8000.0  # MI355X spec, /opt/skills/guides/MI355X_MICROARCH.md (HBM3E 8.0 TB/s)
# measured on MI355X (profiles/r01_copy_style_probe.log, tools/microbench/copy_style_probe.hip): the best
# plain-streaming rates -- one-shot float4 copy (1:1) and a one-shot 4:1 read:write mix (nt loads and
# stores); and the roofline kernel's (the k16 e4 decode apply's) own access pattern with trivial compute:
# per block the 12 received sources and 4 repairs read in slot order, 4 recovered rows written packed,
# one wave per block (profiles/r04_dec_probe_k16.log, tools/microbench/split_probe.hip "dec": 5498-5569
# GB/s at 3 and 4 waves/SIMD; the encode's one-wave pattern on that box 5475-5685)
MEASURED_COPY_GBS = 6282.0
MEASURED_MIX41_GBS = 6440.0
PATTERN_CEILING_GBS = 5530.0
METRIC = "FEC encode+decode GiB/s (device-resident, 1200B symbols)"


def parse():
    p = argparse.ArgumentParser()
    p.add_argument("--gpus", type=int, default=None,
                   help="GPUs (one rank each); default: WORLD_SIZE under a launcher, else 1")
    p.add_argument("--config", choices=["k16", "k32r8", "k64r16"], default="k16",
                   help="workload: k16 = the metric's configs[1]+[2] (default); k32r8 = configs[3] "
                        "(2^24 blocks split over the GPUs); k64r16 = configs[4]")
    p.add_argument("--steps", type=int, default=10)
    p.add_argument("--warmup", type=int, default=3)
    p.add_argument("--blocks", type=int, default=1 << 20, help="FEC blocks per GPU")
    p.add_argument("--k", type=int, default=16)
    p.add_argument("--r", type=int, default=4)
    p.add_argument("--erasures", type=int, default=4)
    p.add_argument("--symbol", type=int, default=1200)
    p.add_argument("--no-legs", action="store_true", help="skip the PCIe and k=32 r=8 encode legs")
    p.add_argument("--no-pcie", action="store_true", help="skip the PCIe end-to-end legs")
    p.add_argument("--cpu-seconds", type=float, default=12.0, help="target CPU-baseline sample time")
    p.add_argument("--no-cpu", action="store_true")
    p.add_argument("--cpu-blocks", type=int, default=0,
                   help="CPU-baseline sample size in blocks (0: about 300 MiB of source payload)")
    p.add_argument("--host-legs", action="store_true", help=argparse.SUPPRESS)  # the child of host_legs_child()
    p.add_argument("--dry-run", action="store_true",
                   help="launcher / rendezvous check without a GPU: ranks time an empty step on gloo; "
                        "value is 0 and the line says dry_run (tests only)")
    a = p.parse_args()
    if a.gpus is None:  # torchrun --nproc-per-node N bench.py: N ranks
        a.gpus = int(os.environ.get("WORLD_SIZE", "1"))
    return a


def traffic_build(kernel_tag: str):
    """Which build and run the committed PMC figure for `kernel_tag` was measured on (its "measured_at")."""
    try:
        with open(os.path.join(ROOT, "profiles", "pmc_traffic.json")) as f:
            return json.load(f).get(kernel_tag, {}).get("measured_at")
    except Exception:
        return None


def load_traffic(kernel_tag: str, blocks: int | None = None):
    """HBM bytes per launch from the committed PMC profile (profiles/pmc_traffic.json), scaled to
    `blocks` when the profile recorded its per-block figure."""
    path = os.path.join(ROOT, "profiles", "pmc_traffic.json")
    if not os.path.exists(path):
        return None
    try:
        with open(path) as f:
            d = json.load(f).get(kernel_tag, {})
        if blocks and d.get("hbm_bytes_per_block_corrected"):
            return float(d["hbm_bytes_per_block_corrected"]) * blocks
        v = d.get("hbm_bytes_per_launch_corrected")
        return float(v) if v else None
    except Exception:
        return None


def make_erasures(torch, nb, k, e, seed, dev):
    """e distinct random source erasures per block; presence masks as [nb, 2] int64 (128 bits)."""
    g = torch.Generator(device="cpu").manual_seed(seed)
    keys = torch.rand((nb, k), generator=g)
    miss = keys.argsort(dim=1)[:, :e]
    pres = torch.ones((nb, 128), dtype=torch.bool)
    pres[:, k:] = False
    pres.scatter_(1, miss, False)
    sp = torch.zeros((nb, 2), dtype=torch.int64)
    for w in range(2):
        bits = pres[:, 64 * w: 64 * w + 64].to(torch.int64)
        lo = (bits[:, :63] << torch.arange(63, dtype=torch.int64)).sum(1)
        sp[:, w] = lo | (bits[:, 63] << 63)  # bit 63 wraps to the sign bit, as a uint64 would
    return sp.to(dev), miss


def check_recovered(torch, dst, src, ok, miss, nb, k, L, what):
    """Decode gate: in every recovered block, the recovered symbols equal the originals.  dst holds
    them packed (fecgpu_rlc_decode_apply_packed: row u of block b = its u-th erased source, ascending),
    one new row per recovered symbol, as the reference's fec_recover allocates each anew."""
    e = miss.shape[1]
    miss = miss.to(src.device).sort(dim=1).values
    em = dst.shape[1]
    for c0 in range(0, nb, 1 << 16):  # chunked: no full-size temporaries
        c1 = min(nb, c0 + (1 << 16))
        b = torch.arange(c0, c1, device=src.device)
        okc = ok[c0:c1].repeat_interleave(e)
        rows = (b.unsqueeze(1) * k + miss[c0:c1]).reshape(-1)[okc]
        drows = (b.unsqueeze(1) * em + torch.arange(e, device=src.device)).reshape(-1)[okc]
        assert bool((dst.view(nb * em, L)[drows] == src.view(nb * k, L)[rows]).all()), what


def encode_kernel_name(k, r, L):
    """The encode kernel the engine's default dispatch runs for (k, r, L) (fec_engine.hip
    fecgpu_rlc_encode): the LDS-ring body for 16-repair tiles (knob ring = 2), else the
    register-prefetch body."""
    rt = 16 if r >= 16 else 8 if r >= 8 else 4 if r >= 4 else 2 if r >= 2 else 1
    vec = 16 if L >= 16 else 8 if L % 8 == 0 else 4
    if rt == 16 and vec == 16 and k >= 4:
        return "k_rlc_encode_bs2<16>"
    return f"k_rlc_encode_bs<{rt},{vec}>"


def apply_kernel_name(k, r, L):
    """The decode data-pass kernel of the default dispatch (fec_engine.hip decode_apply_impl)."""
    em = min(k, r)
    ert = 16 if em > 8 else 8 if em > 4 else 4 if em > 2 else em
    vec = 16 if L >= 16 else 8 if L % 8 == 0 else 4
    if ert == 16 and vec == 16 and k >= 5:
        return "k_rlc_recover_bs2<16>"
    return f"k_rlc_recover_bs<{ert},{vec}>"


def rlc_leg(torch, eng, dev, k, r, L, nb, e, reps=3, seed=0x5EEDF3C0):
    """One BASELINE config as a side leg: RLC encode, then decode with e random erasures,
    device-resident, per-kernel event timing; decode correctness gated on the output."""
    src = torch.empty((nb, k, L), dtype=torch.uint8, device=dev)
    eng.synth_fill(src, src.numel(), seed, 0)
    rep = torch.empty((nb, r, L), dtype=torch.uint8, device=dev)
    work = src.clone()
    sp, miss = make_erasures(torch, nb, k, e, 3, dev)
    idx = (torch.arange(nb, device=dev).unsqueeze(1) * k + miss.to(dev)).reshape(-1)
    work.view(nb * k, L)[idx] = 0xA5
    rp = torch.zeros((nb, 2), dtype=torch.int64, device=dev)
    rp[:, 0] = (1 << r) - 1 if r < 64 else -1
    st = torch.empty(nb, dtype=torch.uint8, device=dev)
    rec = torch.empty((nb, 2), dtype=torch.int64, device=dev)
    ws = eng.alloc_workspace(nb, k, r)
    rec_rows = torch.empty((nb, min(k, r), L), dtype=torch.uint8, device=dev)  # recovered symbols, packed
    stream = torch.cuda.current_stream(dev)
    # one untimed pass, the timed ones straight after it (no host work between them: an idle GPU
    # starts the next kernel at a lower clock), then the gate on the last timed pass's outputs
    eng.rlc_encode(src, rep, k, r, L)
    eng.rlc_decode_stages(work, rep, sp, rp, st, rec, k, r, L, nb, ws, dst=rec_rows, packed=True)
    evs = [[torch.cuda.Event(enable_timing=True) for _ in range(4)] for _ in range(reps)]
    for ev in evs:
        ev[0].record(stream)
        eng.rlc_encode(src, rep, k, r, L)
        eng.rlc_decode_stages(work, rep, sp, rp, st, rec, k, r, L, nb, ws, events=ev[1:], dst=rec_rows, packed=True)
    torch.cuda.synchronize()
    t = [sum(ev[i].elapsed_time(ev[i + 1]) for ev in evs) / reps for i in range(3)]
    ok = st == 0
    check_recovered(torch, rec_rows, src, ok, miss, nb, k, L, f"k{k} r{r} decode did not restore the sources")
    n_rec = int(ok.sum())
    enc_b, app_b = (k + r) * L * nb, (k + e) * L * n_rec
    del src, rep, work, ws, rec_rows
    torch.cuda.empty_cache()
    pay = nb * k * L / 2**30
    return {"blocks": nb, "k": k, "r": r, "L": L, "erasures": e, "encode_kernel": encode_kernel_name(k, r, L),
            "apply_kernel": apply_kernel_name(k, r, L),
            "encode_ms": round(t[0], 3),
            "plan_ms": round(t[1], 3), "apply_ms": round(t[2], 3),
            "payload_GiB_s": round(pay / ((t[0] + t[1] + t[2]) * 1e-3), 2),
            "encode_GB_s": round(enc_b / (t[0] * 1e-3) / 1e9, 1),
            "encode_hbm_frac": round(enc_b / (t[0] * 1e-3) / 1e9 / HBM_PEAK_GBS, 4),
            "apply_GB_s": round(app_b / (t[2] * 1e-3) / 1e9, 1),
            "recovered_blocks": n_rec, "ref_ub_blocks": int((st == 2).sum())}


def xor_leg(torch, eng, dev, k, L, nb, reps=3):
    """XOR scheme (configs[0]'s scheme at GPU scale): encode, then recover one erasure per block into a
    row of its own (fecgpu_xor_decode_to; the reference's fec_recover allocates the recovered symbol
    anew, xor_fec_scheme.c:54-58; in place into the received block measured 8 % slower,
    profiles/r03_ab_xor_decode_to.log)."""
    src = torch.empty((nb, k, L), dtype=torch.uint8, device=dev)
    eng.synth_fill(src, src.numel(), 0x5EEDF3C0, 0)
    rep = torch.empty((nb, 1, L), dtype=torch.uint8, device=dev)
    work = src.clone()
    sp, miss = make_erasures(torch, nb, k, 1, 4, dev)
    idx = (torch.arange(nb, device=dev).unsqueeze(1) * k + miss.to(dev)).reshape(-1)
    work.view(nb * k, L)[idx] = 0xA5
    rp = torch.ones((nb, 2), dtype=torch.int64, device=dev)
    rp[:, 1] = 0
    st = torch.empty(nb, dtype=torch.uint8, device=dev)
    rec = torch.empty((nb, 2), dtype=torch.int64, device=dev)
    dst = torch.empty((nb, L), dtype=torch.uint8, device=dev)
    stream = torch.cuda.current_stream(dev)
    # untimed pass, timed passes back to back, then the gate (as rlc_leg)
    eng.xor_encode(src, rep, k, L)
    eng.xor_decode_to(work, rep, dst, sp, rp, st, rec, k, L)
    evs = [[torch.cuda.Event(enable_timing=True) for _ in range(3)] for _ in range(reps)]
    for ev in evs:
        ev[0].record(stream)
        eng.xor_encode(src, rep, k, L)
        ev[1].record(stream)
        eng.xor_decode_to(work, rep, dst, sp, rp, st, rec, k, L)
        ev[2].record(stream)
    torch.cuda.synchronize()
    te = sum(ev[0].elapsed_time(ev[1]) for ev in evs) / reps
    td = sum(ev[1].elapsed_time(ev[2]) for ev in evs) / reps
    assert bool((st == 0).all()) and bool((dst == src.view(nb * k, L)[idx]).all()), \
        "xor decode did not restore the sources"
    del src, rep, work, dst
    torch.cuda.empty_cache()
    pay = nb * k * L / 2**30
    return {"blocks": nb, "k": k, "L": L, "decode_output": "recovered symbol into a row of its own per block",
            "encode_ms": round(te, 3), "decode_ms": round(td, 3),
            "payload_GiB_s": round(pay / ((te + td) * 1e-3), 2),
            "encode_GB_s": round((k + 1) * L * nb / (te * 1e-3) / 1e9, 1),
            "decode_GB_s": round((k + 1) * L * nb / (td * 1e-3) / 1e9, 1)}


def host_cpu_share():
    """CPUs this process may use: the affinity mask, bounded by a cgroup CPU quota when one is set
    (a GPU box shares its host: its affinity mask can list every CPU of the machine while the
    quota grants a slice of them)."""
    aff = len(os.sched_getaffinity(0))
    quota = None
    try:
        with open("/sys/fs/cgroup/cpu.max") as f:
            q, per = f.read().split()[:2]
        if q != "max":
            quota = int(q) / int(per)
    except (OSError, ValueError):
        pass
    cores = aff if quota is None else max(1, min(aff, int(quota + 0.5)))
    return cores, aff, quota


def cpu_baseline(args, ncores, k, r, e, L):
    """The reference's own plugins/fec scheme pluglets (rlc_fec_scheme_generate_gf256.c,
    rlc_fec_scheme_gf256.c compiled natively from the reference sources into
    oracle/_ref/libfecref.so; kind "reference") on every core of this process's CPU share, one
    fork()ed worker per core, over a bounded sample of the same workload: RLC encode of every
    block, then (e > 0) decode with e erasures.  The reference segfaults on ~1-5 % of erasure
    patterns; those blocks are screened out of its decode (untimed, by the CPU
    port) and the value still counts their payload, so the reference number is, if anything,
    flattering.  The port (oracle/fec_oracle.c, bit-exact) is timed beside it on as many threads;
    their ratio is reported.  Runs before the process touches the GPU (the workers are forks)."""
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import ctypes as C
    import numpy as np
    from oracle_py import Oracle, synth_bytes
    o = Oracle()
    nb = args.cpu_blocks or max(16, (300 << 20) // (k * L))  # ~300 MiB of payload: beyond the host caches
    src = synth_bytes(nb * k * L, 0x5EEDF3C0).reshape(nb, k, L)
    rng = np.random.default_rng(1)
    sp = np.zeros((nb, 2), np.uint64)
    rp = np.zeros((nb, 2), np.uint64)
    for b in range(nb):
        m = [(1 << min(k, 64)) - 1, (1 << max(k - 64, 0)) - 1]
        for j in (rng.choice(k, e, replace=False) if e else ()):
            m[int(j) >> 6] &= ~(1 << (int(j) & 63))
        sp[b] = m
        rp[b] = [(1 << min(r, 64)) - 1, (1 << max(r - 64, 0)) - 1]
    if e:  # screen: which patterns the reference survives (the port flags its x[-1] crash exactly)
        rep0 = o.rlc_encode_batch(src, r, 0, ncores)
        st, _ = o.rlc_decode_batch(src.copy(), rep0, sp, rp, 0, ncores)
        skip = (st == 2).astype(np.uint8)
        del rep0
    else:  # encode-only workload: every block skips the reference's decode half
        skip = np.ones(nb, np.uint8)
    what = f"RLC encode{' + decode' if e else ''} pluglets"
    out = {"unit": "GiB/s", "cores": ncores, "kind": "reference"}
    ref_path = os.path.join(ROOT, "oracle", "_ref", "libfecref.so")
    gib_pass = nb * k * L / 2**30
    if os.path.exists(ref_path):
        lib = C.CDLL(ref_path)
        lib.ref_cpu_baseline.argtypes = [C.c_int, C.c_void_p, C.c_uint64, C.c_int, C.c_int, C.c_int, C.c_uint32,
                                         C.c_void_p, C.c_void_p, C.c_int, C.POINTER(C.c_double)]
        res = (C.c_double * 3)()
        assert lib.ref_cpu_baseline(ncores, src.ctypes.data, nb, k, r, L, 0, sp.ctypes.data, skip.ctypes.data, 1,
                                    res) == 0, "reference CPU workers failed"
        passes = max(1, min(200, int(round(args.cpu_seconds / max(res[0], 1e-3)))))
        assert lib.ref_cpu_baseline(ncores, src.ctypes.data, nb, k, r, L, 0, sp.ctypes.data, skip.ctypes.data,
                                    passes, res) == 0, "reference CPU workers failed"
        out["value"] = round(passes * gib_pass / res[0], 4)
        out["sample"] = (f"{passes} passes x {nb} blocks, k={k} r={r} e={e} L={L}: the reference's {what} "
                         f"(native gcc -O2), {ncores} fork()ed workers, {res[0]:.1f} s wall"
                         + (f"; {int(skip.sum())} of {nb} erasure patterns crash the reference and are not decoded"
                            if e else ""))
    else:  # the reference build is absent: the port stands in (and says so)
        out["kind"] = "port"
    # the port on the same sample and thread count (second number, and its ratio to the reference)
    passes_p, t_total = 0, 0.0
    while t_total < args.cpu_seconds / 2 and passes_p < 1000:
        work = src.copy()
        t0 = time.perf_counter()
        rep = o.rlc_encode_batch(work, r, 0, ncores)
        if e:
            o.rlc_decode_batch(work, rep, sp, rp, 0, ncores)
        t_total += time.perf_counter() - t0
        passes_p += 1
    port = round(passes_p * gib_pass / t_total, 4)
    out["port"] = {"value": port, "threads": ncores,
                   "sample": f"{passes_p} passes x {nb} blocks, oracle/fec_oracle.c -O2, {t_total:.1f} s"}
    if "value" in out:
        out["port"]["port_over_reference"] = round(port / out["value"], 3)
    else:
        out["value"] = port
        out["sample"] = out["port"]["sample"]
    return out


def workload_cfg(args):
    cfg = dict(CONFIGS[args.config])
    if args.config == "k16":  # the legacy flags still shape the default workload
        cfg.update(k=args.k, r=args.r, e=args.erasures, L=args.symbol, per_rank=args.blocks)
    return cfg


def measure_cpu_baseline(args, cfg):
    """cpu_baseline for this workload (computed once per job, before any process touches the GPU)."""
    ncores, aff, quota = host_cpu_share()
    cpu = cpu_baseline(args, ncores, cfg["k"], cfg["r"], cfg["e"], cfg["L"])
    cpu["host"] = {"affinity_cpus": aff, "cgroup_quota_cpus": quota}
    return cpu


def _free_port():
    import socket
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def visible_gpu_count(timeout=300):
    """GPUs a child rank could open, counted in a throw-away child process: whatever the count costs
    (HIP initialisation, /dev/kfd) happens there, and the launcher itself never opens the device."""
    import subprocess
    code = "import torch; print(torch.cuda.device_count())"
    try:
        p = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True, timeout=timeout)
        return int(p.stdout.strip().splitlines()[-1]) if p.returncode == 0 else 0
    except (subprocess.TimeoutExpired, ValueError, IndexError):
        return 0


def gpu_device_fds():
    """Open file descriptors of this process on a GPU device node (/dev/kfd, /dev/dri/*)."""
    out = []
    try:
        for fd in os.listdir("/proc/self/fd"):
            try:
                t = os.readlink(f"/proc/self/fd/{fd}")
            except OSError:
                continue
            if t == "/dev/kfd" or t.startswith("/dev/dri/"):
                out.append(t)
    except OSError:
        pass
    return out


def launch_ranks(args):
    """`bench.py --gpus N` run directly (no WORLD_SIZE in the environment): this process never touches
    the GPU.  It counts the GPUs in a throw-away child (visible_gpu_count), then starts N child processes
    of this script, one per GPU (RANK = LOCAL_RANK = i, WORLD_SIZE = N, rendezvous on 127.0.0.1), waits for
    all of them and exits with the first failure's code.  cpu_baseline is an N = 1 figure (measured by
    rank 0 of a one-GPU run only), so an N > 1 line carries none.  Rank 0 prints the JSON line.  No exec: the
    children are started as new processes, and the launcher checks it holds no GPU device open first."""
    import signal
    import subprocess
    import tempfile
    n = args.gpus
    if not args.dry_run and os.environ.get("PQUIC_BENCH_SHARE_GPU") != "1":
        have = visible_gpu_count()
        if have < n:
            print(f"bench.py: --gpus {n} but {have} GPU(s) visible", file=sys.stderr)
            return 2
    held = gpu_device_fds()
    if held:  # a parent that initialised the GPU must not start the ranks (forks of a HIP process)
        print(f"bench.py: launcher holds GPU device files open ({', '.join(held)}); refusing to start ranks",
              file=sys.stderr)
        return 3
    cfg = workload_cfg(args)
    env = dict(os.environ)
    tmp = None
    if not args.no_cpu and n == 1:  # never, here (n > 1): kept for a launcher of one rank
        cpu = measure_cpu_baseline(args, cfg)
        fd, tmp = tempfile.mkstemp(prefix="pquic_bench_cpu_", suffix=".json")
        with os.fdopen(fd, "w") as f:
            json.dump(cpu, f)
        env["PQUIC_BENCH_CPU_JSON"] = tmp
    env.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(_free_port()), WORLD_SIZE=str(n),
               LOCAL_WORLD_SIZE=str(n), PQUIC_BENCH_LAUNCHED="1")
    procs = []
    try:
        for i in range(n):
            env_i = dict(env, RANK=str(i), LOCAL_RANK=str(i))
            procs.append(subprocess.Popen([sys.executable, os.path.abspath(__file__)] + sys.argv[1:], env=env_i))
        rc = 0
        live = list(procs)
        while live:
            for p in list(live):
                c = p.poll()
                if c is None:
                    continue
                live.remove(p)
                if c != 0 and rc == 0:
                    rc = c if c > 0 else 128 - c
                    for q in live:  # one rank failed: the others would wait at a barrier forever
                        q.send_signal(signal.SIGTERM)
            time.sleep(0.05)
        return rc
    finally:
        for p in procs:
            if p.poll() is None:
                p.kill()
                p.wait()
        if tmp:
            os.unlink(tmp)


def pcie_legs(torch, args, dev):
    """End-to-end rate from / to pinned host buffers (H2D + kernels + D2H, overlapped on 3
    streams).  Reported beside, never as, the device-resident value."""
    from pquic_amd import HostPath
    nb, k, r, L, e = 1 << 18, args.k, args.r, args.symbol, args.erasures
    hp = HostPath(dev.index or 0, 3, 64 << 20)
    src = torch.empty((nb, k, L), dtype=torch.uint8, pin_memory=True)
    src.copy_(torch.randint(0, 256, (nb, k, L), dtype=torch.uint8))
    rep = torch.empty((nb, r, L), dtype=torch.uint8, pin_memory=True)
    sp, _ = make_erasures(torch, nb, k, e, 5, "cpu")
    sp = sp.pin_memory()
    rp = torch.zeros((nb, 2), dtype=torch.int64).pin_memory()
    rp[:, 0] = (1 << r) - 1
    st = torch.empty(nb, dtype=torch.uint8, pin_memory=True)
    rec = torch.empty((nb, 2), dtype=torch.int64, pin_memory=True)
    hp.rlc_encode(src, rep, nb, k, r, L)
    t0 = time.perf_counter()
    for _ in range(3):
        hp.rlc_encode(src, rep, nb, k, r, L)
    t_enc = (time.perf_counter() - t0) / 3
    hp.rlc_decode(src, rep, sp, rp, st, rec, nb, k, r, L)
    t0 = time.perf_counter()
    for _ in range(3):
        hp.rlc_decode(src, rep, sp, rp, st, rec, nb, k, r, L)
    t_dec = (time.perf_counter() - t0) / 3
    hp.close()
    pay = nb * k * L / 2**30
    return {"pcie_e2e_encode_k16_r4": {"blocks": nb, "payload_GiB_s": round(pay / t_enc, 2),
                                       "pcie_GB_s": round((k + r) * L * nb / t_enc / 1e9, 1)},
            "pcie_e2e_decode_k16_e4": {"blocks": nb, "payload_GiB_s": round(pay / t_dec, 2),
                                       "pcie_GB_s": round((k + r + e) * L * nb / t_dec / 1e9, 1),
                                       "note": "pinned host buffers: block rows H2D, recovered rows written "
                                               "by the apply kernel straight into host memory"}}


def batching_legs(dev_index, args):
    """§8f row 1: the block framework's blocks through the batching adapter
    (include/pquic_fec_batch.h), end to end from host packet buffers: PCIe, kernels, completion on the
    caller thread.  tools/batch_load.c plays the single-threaded sender (or receiver) over 64 or 512
    connections, each with its own 16 MiB plugin arena (PLUGIN_MEMORY, picoquic_internal.h:523,576; one
    plugin instance per connection, plugin.c:835,946-950) holding its symbols.  Registered arenas
    (pquic_fec_batch_register_heap, one per connection): the kernels read sources / received symbols
    and write repairs / recovered symbols in place; "staged": unregistered, the stager threads copy every
    row through pinned staging.  A sender keeps at most 3 batches of 2048 blocks in flight (the
    back-pressure that bounds the queueing latency)."""
    import ctypes as C
    path = os.path.join(ROOT, "tools", "libbatchload.so")
    if not os.path.exists(path):
        return {}
    lib = C.CDLL(path)
    D = C.POINTER(C.c_double)
    lib.bl_run.argtypes = [C.c_int, C.c_int, C.c_int, C.c_int, C.c_int, C.c_long, C.c_uint, C.c_uint, C.c_int,
                           C.c_double, C.c_int, D]
    lib.bl_run_recover.argtypes = [C.c_int, C.c_int, C.c_int, C.c_int, C.c_int, C.c_int, C.c_long, C.c_uint,
                                   C.c_uint, C.c_int, C.c_int, D]
    lib.bl_run_window.argtypes = [C.c_int, C.c_int, C.c_int, C.c_int, C.c_int, C.c_int, C.c_long, C.c_uint,
                                  C.c_uint, C.c_int, C.c_int, D]
    lib.bl_run_senders.argtypes = [C.c_int] + lib.bl_run.argtypes[:9] + [C.c_int, D]
    lib.bl_set_inflight.argtypes = [C.c_int]
    lib.bl_last_rows.argtypes = [D]
    lib.bl_last_latency.argtypes = [D]
    lib.bl_last_jobs.argtypes = [D]
    REG, PER_CONN = 1, 2
    batch, inflight = 2048, 3
    lib.bl_set_inflight(inflight)
    legs = {}

    def median_of(runs, fn):
        """host-side rates on a shared CPU slice vary from run to run: the run with the median rate"""
        res = []
        for _ in range(runs):
            out, rows, q, jb = (C.c_double * 8)(), (C.c_double * 2)(), (C.c_double * 8)(), (C.c_double * 3)()
            rc = fn(out)
            if rc:
                return rc, None, None
            lib.bl_last_rows(rows)
            lib.bl_last_latency(q)
            lib.bl_last_jobs(jb)
            res.append((list(out), list(rows), list(q), list(jb)))
        res.sort(key=lambda x: x[0][0])
        out, rows, q, jb = res[len(res) // 2]
        return 0, out, {"runs_payload_GiB_s": [round(o[0][0], 2) for o in res],
                        "runs_latency_us_p99": [o[0][2] for o in res], "rows_in_place": int(rows[0]),
                        "rows_staged": int(rows[1]), "latency_us_p90": q[1], "latency_us_p99_9": q[4],
                        "jobs_allocated_on_sender_thread": int(jb[0]),
                        "job_alloc_ms_on_sender_thread": round(jb[1] / 1000.0, 2),
                        "polls_holding_for_a_job": int(jb[2])}

    def leg(out, extra, **kw):
        d = {"k": args.k, "r": args.r, "L": args.symbol, "batch_blocks": batch, "batches_in_flight": inflight,
             "max_delay_us": 2000}
        d.update(kw)
        d.update({"payload_GiB_s": round(out[0], 2), "latency_us_p50": out[1], "latency_us_p99": out[2],
                  "latency_us_max": out[3], "batches": int(out[4]), "mean_blocks_per_batch": round(out[7], 1)})
        d.update(extra)
        return d

    # one short untimed sender run first: the process's one-time costs (the engine's first launches and
    # host contexts, the allocator's first page faults, thread start-up) land outside the measured legs
    warm = (C.c_double * 8)()
    lib.bl_run(dev_index, args.k, args.r, args.symbol, 64, 20000, batch, 2000, 2, 0.0, REG | PER_CONN, warm)
    for name, nconn, reg, runs in (("saturated", 64, REG | PER_CONN, 3), ("saturated_512conn", 512, REG | PER_CONN, 3),
                                   ("saturated_staged", 64, PER_CONN, 3)):
        rc, out, extra = median_of(runs, lambda o: lib.bl_run(dev_index, args.k, args.r, args.symbol, nconn, 200000,
                                                              batch, 2000, 2, 0.0, reg, o))
        legs["batch_" + name] = {"error": rc} if rc else leg(
            out, extra, blocks=200000, connections=nconn, arenas="one 16 MiB arena per connection",
            rows="in place (registered arenas)" if reg & REG else "staged by copies", source_pool_blocks=32768)
    rc, out, extra = median_of(3, lambda o: lib.bl_run_recover(dev_index, args.k, args.r, args.symbol, args.erasures,
                                                               64, 200000, batch, 2000, 2, REG | PER_CONN, o))
    legs["batch_recover_saturated"] = {"error": rc} if rc else leg(
        out, extra, blocks=200000, connections=64, erasures=args.erasures, recovered_symbols=int(out[6]),
        arenas="one 16 MiB arena per connection",
        rows="received symbols read and recovered symbols written in place (registered arenas; recovered "
             "symbols allocated at submission)", source_pool_blocks=32768)
    rc, out, extra = median_of(1, lambda o: lib.bl_run_recover(dev_index, args.k, args.r, args.symbol, args.erasures,
                                                               64, 200000, batch, 2000, 2, PER_CONN, o))
    legs["batch_recover_saturated_staged"] = {"error": rc} if rc else leg(
        out, extra, blocks=200000, connections=64, erasures=args.erasures, recovered_symbols=int(out[6]),
        rows="staged by copies")
    rc, out, extra = median_of(1, lambda o: lib.bl_run(dev_index, args.k, args.r, args.symbol, 64, 100000, 4096, 250,
                                                       2, 2.0, REG | PER_CONN, o))
    legs["batch_paced_2GiBps"] = {"error": rc} if rc else leg(
        out, extra, blocks=100000, connections=64, offered_GiB_s=2.0, max_delay_us=250, batch_blocks=4096)
    # two sender threads, each with its own batcher and 64 connections: a server running one
    # single-threaded PQUIC process per core on one GPU (one sender alone is bound by its own thread).
    # Two batchers share the GPU, so each takes half the batch: the same rate at half the latency
    # (profiles/r05_senders_sweep.log: 2048 blocks 48.0 GiB/s at p99 5.1-6.9 ms, 1024 46.6 at 2.7-3.1 ms)
    batch2 = 1024
    res = []
    for _ in range(3):
        out = (C.c_double * 8)()
        if lib.bl_run_senders(2, dev_index, args.k, args.r, args.symbol, 64, 200000, batch2, 2000, 2,
                              REG | PER_CONN, out):
            break
        res.append(list(out))
    if len(res) == 3:
        out = sorted(res, key=lambda o: o[0])[1]
        legs["batch_saturated_2senders"] = leg(
            out, {"runs_payload_GiB_s": [round(o[0], 2) for o in res]}, batch_blocks=batch2, senders=2,
            blocks_per_sender=200000,
            connections_per_sender=64, arenas="one 16 MiB arena per connection",
            note="both senders start each pass at a barrier; rate = all blocks over first start to last drain; "
                 "latency = the worse sender's percentile")
    else:
        legs["batch_saturated_2senders"] = {"error": -1}
    lib.bl_set_inflight(4)
    # the sliding-window sender (window_framework_sender.h:209-260) at the redundancy controllers'
    # shapes: a window of the <= 30 symbols in flight every K new ones, N - K repairs
    # batches of 1536 windows: the same or a higher rate than 2048 or 4096, at a third of 4096's p99
    # (profiles/r05_window_batch_sweep.log)
    wbatch = 1536
    for k, r, step in ((30, 1, 5), (30, 5, 25)):
        leg_w = {"k": k, "r": r, "L": args.symbol, "step": step, "windows": 200000, "connections": 64,
                 "batch_blocks": wbatch, "max_delay_us": 2000}
        for api, tag in ((1, "window_api"), (0, "block_api")):
            out = (C.c_double * 8)()
            rc = lib.bl_run_window(dev_index, k, r, args.symbol, step, 64, 200000, wbatch, 2000, 2, api, out)
            leg_w[tag] = {"error": rc} if rc else {
                "stream_GiB_s": round(out[0], 2), "window_GiB_s": round(out[7], 2), "latency_us_p50": out[1],
                "latency_us_p99": out[2], "batches": int(out[4])}
        legs[f"batch_window_k{k}_r{r}_step{step}"] = leg_w
    return legs


def hook_latency_legs(dev_index):
    """Latency of the synchronous drop-in hooks (one block per call, the way the block framework
    calls fec_generate_repair_symbols / fec_recover; tools/batch_load.c bl_hook_latency) at k16 r4
    L1200 with 4 erasures, next to the reference pluglets' own time per block on one core of this
    box (oracle/_ref/libfecref.so, in process)."""
    import ctypes as C
    path = os.path.join(ROOT, "tools", "libbatchload.so")
    if not os.path.exists(path):
        return {}
    lib = C.CDLL(path)
    lib.bl_hook_latency.argtypes = [C.c_int, C.c_int, C.c_int, C.c_int, C.c_int, C.c_long, C.POINTER(C.c_double)]
    out = (C.c_double * 7)()
    rc = lib.bl_hook_latency(dev_index, 16, 4, 1200, 4, 2000, out)
    if rc:
        return {"sync_hook_k16_r4": {"error": rc}}
    leg = {"k": 16, "r": 4, "L": 1200, "erasures": 4, "calls": 2000,
           "generate_us_p50": out[0], "generate_us_p99": out[1], "generate_us_mean": round(out[2], 1),
           "recover_us_p50": out[3], "recover_us_p99": out[4], "recover_us_mean": round(out[5], 1),
           "recovered_per_call": out[6]}
    # the same hooks while a bulk job (4096-block k16 r4 encodes from page-locked memory, back to back:
    # the batching adapter's kind of kernel) occupies the GPU; the resident service withdraws a request
    # it could not serve within 2 ms and the call takes the launch path
    lib.bl_hook_latency_loaded.argtypes = [C.c_int, C.c_int, C.c_long, C.POINTER(C.c_double)]
    lib.bl_bulk_rate.argtypes = [C.c_int, C.c_int, C.c_int, C.POINTER(C.c_double)]
    alone = (C.c_double * 2)()
    rc_alone = lib.bl_bulk_rate(dev_index, 4096, 200, alone)  # the bulk call with no hooks, same run
    lo = (C.c_double * 11)()
    rc = lib.bl_hook_latency_loaded(dev_index, 4096, 2000, lo)
    leg["under_bulk_load"] = {"error": rc} if rc else {
        "bulk": "fecgpu_rlc_encode_host, 4096 blocks k16 r4 L1200 per call, page-locked, back to back",
        "generate_us_p50": lo[0], "generate_us_p99": lo[1], "recover_us_p50": lo[3], "recover_us_p99": lo[4],
        "bulk_calls_meanwhile": int(lo[7]), "bulk_ms_per_call_mean": round(lo[9], 3),
        "bulk_ms_per_call_max": round(lo[10], 3), "requests_withdrawn_at_deadline": int(lo[8])}
    if not rc and not rc_alone:
        leg["under_bulk_load"]["bulk_alone_ms_per_call"] = round(alone[0], 3)
        leg["under_bulk_load"]["bulk_beside_hooks_over_alone"] = round(lo[9] / alone[0], 3)
        # the same without slicing (knob yield_slice_kb 0): what the slices buy, and what they cost
        eng = C.CDLL(os.path.join(ROOT, "pquic_amd", "lib", "libpquic_fec.so"))
        eng.fecgpu_set_knob.argtypes = [C.c_char_p, C.c_int]
        eng.fecgpu_get_knob.argtypes = [C.c_char_p, C.POINTER(C.c_int)]
        kb = C.c_int(0)
        un = (C.c_double * 11)()
        if eng.fecgpu_get_knob(b"yield_slice_kb", C.byref(kb)) == 0 and eng.fecgpu_set_knob(b"yield_slice_kb", 0) == 0:
            try:
                if lib.bl_hook_latency_loaded(dev_index, 4096, 2000, un) == 0:
                    leg["under_bulk_load"]["unsliced"] = {
                        "generate_us_p99": un[1], "recover_us_p99": un[4], "bulk_ms_per_call_mean": round(un[9], 3),
                        "bulk_beside_hooks_over_alone": round(un[9] / alone[0], 3)}
            finally:
                eng.fecgpu_set_knob(b"yield_slice_kb", kb.value)
    ref_path = os.path.join(ROOT, "oracle", "_ref", "libfecref.so")
    if os.path.exists(ref_path):
        sys.path.insert(0, os.path.join(ROOT, "oracle"))
        import numpy as np
        from oracle_py import Oracle, synth_bytes
        nb, k, r, L = 2000, 16, 4, 1200
        src = synth_bytes(nb * k * L, 7).reshape(nb, k, L)
        sp = np.zeros((nb, 2), np.uint64)
        for b in range(nb):
            first = b % (k - 3)
            sp[b, 0] = ((1 << k) - 1) & ~(0xF << first)
        rp = np.zeros((nb, 2), np.uint64)
        rp[:, 0] = (1 << r) - 1
        o = Oracle()
        st, _ = o.rlc_decode_batch(src.copy(), o.rlc_encode_batch(src, r, 0, 1), sp, rp, 0, 1)
        skip = (st == 2).astype(np.uint8)
        rl = C.CDLL(ref_path)
        rl.ref_work_serial.restype = C.c_long
        rl.ref_work_serial.argtypes = [C.c_void_p, C.c_uint64, C.c_int, C.c_int, C.c_int, C.c_uint32, C.c_void_p,
                                       C.c_void_p, C.POINTER(C.c_double), C.POINTER(C.c_double)]
        te, td = C.c_double(0), C.c_double(0)
        nd = rl.ref_work_serial(src.ctypes.data, nb, k, r, L, 0, sp.ctypes.data, skip.ctypes.data, C.byref(te),
                                C.byref(td))
        if nd > 0:
            leg["reference_pluglet_us_per_block_1core"] = {"generate": round(te.value / nb * 1e6, 1),
                                                           "recover": round(td.value / nd * 1e6, 1)}
    return {"sync_hook_k16_r4": leg}


# Workloads (BASELINE.json configs).  The default is the metric's own configuration (configs[1] +
# configs[2]: k16 r4 encode then 4-erasure decode, 2^20 blocks per GPU).  The others are the
# configs that name 8 GPUs, for multi-GPU runs: configs[3] (k32 r8 encode, 2^24 blocks sharded over
# the GPUs, strong scaling) and configs[4] (k64 r16 L9000 encode + 16-erasure decode, 2^16 blocks
# per GPU).
CONFIGS = {
    "k16": {"k": 16, "r": 4, "e": 4, "L": 1200, "per_rank": 1 << 20, "scaling": "weak",
            "workload": "RLC-GF(256) encode k=16 r=4 + decode 4 erasures, 1200B symbols (configs[1]+[2])"},
    "k32r8": {"k": 32, "r": 8, "e": 0, "L": 1200, "total": 1 << 24, "resident": 1 << 21, "scaling": "strong",
              "workload": "RLC-GF(256) encode k=32 r=8, 1200B symbols, 2^24 blocks split over the GPUs (configs[3])"},
    "k64r16": {"k": 64, "r": 16, "e": 16, "L": 9000, "per_rank": 1 << 16, "scaling": "weak",
               "workload": "RLC-GF(256) encode k=64 r=16 + decode 16 erasures, 9000B symbols (configs[4])"},
}


def rank_device(local):
    """The GPU a rank drives: its LOCAL_RANK (one process per GPU).  PQUIC_BENCH_SHARE_GPU=1 (rehearsal
    on a box with fewer GPUs than ranks, never set by the driver) folds ranks onto the devices present;
    counting devices does not initialise HIP on this image."""
    if os.environ.get("PQUIC_BENCH_SHARE_GPU") == "1":
        import torch
        return local % max(torch.cuda.device_count(), 1)
    return local


def dry_run_rank(args, world, rank, local, cpu):
    """--dry-run: the rank plumbing without a GPU (gloo): barrier, an empty timed region,
    max-over-ranks and per-rank gather (step time and the device each rank would drive), then rank 0's
    line with value 0."""
    import torch
    import torch.distributed as dist
    if world > 1:
        dist.init_process_group("gloo")
        dist.barrier()
    t0 = time.perf_counter()
    elapsed = time.perf_counter() - t0
    per_rank, devices = None, [rank_device(local)]
    if world > 1:
        dist.barrier()
        t = torch.tensor([elapsed], dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        allr = [torch.zeros(1, dtype=torch.float64) for _ in range(world)]
        dist.all_gather(allr, torch.tensor([elapsed], dtype=torch.float64))
        per_rank = [float(x.item()) for x in allr]
        alld = [torch.zeros(1, dtype=torch.int64) for _ in range(world)]
        dist.all_gather(alld, torch.tensor([devices[0]], dtype=torch.int64))
        devices = [int(x.item()) for x in alld]
    if rank == 0:
        print(json.dumps({"metric": METRIC, "value": 0.0, "unit": "GiB/s", "n_gpus": world, "steps": args.steps,
                          "warmup": args.warmup, "dry_run": True, "cpu_baseline": cpu,
                          "per_rank_ms_per_step": per_rank, "per_rank_device": devices}))
    if world > 1:
        dist.barrier()
        dist.destroy_process_group()


def host_legs_child(args, dev_index):
    """The batching-adapter and synchronous-hook legs in a child process of their own: a PQUIC process
    holds the FEC library, not torch and the bench's 50 GB of device tensors, and in the bench's own process
    one sender measured 20 % slower than in a fresh one on the same box (profiles/r05_batch_context_probe.log).
    The child is a plain `python bench.py --host-legs` (no torch import); its JSON line is merged here."""
    import subprocess
    cmd = [sys.executable, os.path.abspath(__file__), "--host-legs", "--k", str(args.k), "--r", str(args.r),
           "--symbol", str(args.symbol), "--erasures", str(args.erasures)]
    env = dict(os.environ)
    env["PQUIC_BENCH_HOST_DEVICE"] = str(dev_index)
    try:
        r = subprocess.run(cmd, capture_output=True, text=True, timeout=600, env=env)
    except subprocess.TimeoutExpired:
        return {"host_legs": {"error": "timeout"}}
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    if r.returncode or not lines:
        return {"host_legs": {"error": r.returncode, "stderr": r.stderr[-2000:]}}
    return json.loads(lines[-1])


def main():
    args = parse()
    if args.host_legs:  # child of host_legs_child: no torch, the engine library and the load generator only
        dev_index = int(os.environ.get("PQUIC_BENCH_HOST_DEVICE", "0"))
        legs = batching_legs(dev_index, args)
        legs.update(hook_latency_legs(dev_index))
        print(json.dumps(legs), flush=True)
        return
    if "WORLD_SIZE" not in os.environ and args.gpus > 1:
        sys.exit(launch_ranks(args))  # parent: starts one child process per GPU, never touches a GPU
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus:
        print(f"bench.py: --gpus {args.gpus} but WORLD_SIZE={world}: launch one process per GPU "
              f"(torchrun --nproc-per-node {args.gpus}, or plain `python bench.py --gpus {args.gpus}`)",
              file=sys.stderr)
        sys.exit(2)
    cfg = workload_cfg(args)
    k, r, e, L = cfg["k"], cfg["r"], cfg["e"], cfg["L"]
    cpu = None
    if rank == 0 and not args.no_cpu and world == 1:  # the CPU baseline is timed at N = 1 only
        path = os.environ.get("PQUIC_BENCH_CPU_JSON")
        if path:  # measured by the launcher before it started the ranks
            with open(path) as f:
                cpu = json.load(f)
        else:  # before any HIP call: the reference's workers are fork()ed from this process
            cpu = measure_cpu_baseline(args, cfg)
    if args.dry_run:
        dry_run_rank(args, world, rank, local, cpu)
        return
    import torch
    from pquic_amd import Engine

    dist = None
    # rehearsal knobs for a box with fewer GPUs than ranks (never set by the driver):
    # PQUIC_BENCH_SHARE_GPU=1 maps rank -> device local % count, PQUIC_BENCH_BACKEND=gloo
    # because RCCL refuses two ranks on one device
    backend = os.environ.get("PQUIC_BENCH_BACKEND", "nccl")
    local = rank_device(local)
    if world > 1:
        import torch.distributed as dist
        torch.cuda.set_device(local)
        dist.init_process_group(backend)
    dev = torch.device(f"cuda:{local}")
    torch.cuda.set_device(dev)
    eng = Engine(local)

    from pquic_amd.shard import fbn_base_of, shard_range, weak_range
    if cfg["scaling"] == "weak":
        g0, g1 = weak_range(cfg["per_rank"], rank)  # this rank's global block range
    else:
        g0, g1 = shard_range(cfg["total"], world, rank)
    share = g1 - g0                                  # blocks this rank codes per step
    nb = min(share, cfg.get("resident", share))      # blocks resident in HBM
    passes = (share + nb - 1) // nb if nb else 0     # a share larger than HBM runs in passes
    src = torch.empty((nb, k, L), dtype=torch.uint8, device=dev)
    eng.synth_fill(src, src.numel(), 0x5EEDF3C0, g0 * k * L)
    rep = torch.empty((nb, r, L), dtype=torch.uint8, device=dev)
    if e:
        work = torch.empty_like(src)
        sp, miss = make_erasures(torch, nb, k, e, 11 + rank, dev)
        rp = torch.zeros((nb, 2), dtype=torch.int64, device=dev)
        rp[:, 0] = (1 << r) - 1 if r < 64 else -1
        status = torch.empty(nb, dtype=torch.uint8, device=dev)
        recovered = torch.empty((nb, 2), dtype=torch.int64, device=dev)
        ws = eng.alloc_workspace(nb, k, r)
        # decode input: the received block (erased slots hold stale bytes), copied once.  The recovered
        # symbols go to their own rows -- the reference's fec_recover allocates every recovered source
        # symbol anew rather than writing into the received block (rlc_fec_scheme_gf256.c:218-236) --
        # packed per block (row u = the u-th erased source): in place measured 5 % slower
        # (profiles/r01_ab_apply_to.log), rows at their src-layout slots 2.3 % slower than packed
        # (profiles/r03_ab_apply_packed.log: each leaves two half-written 128-B lines)
        work.copy_(src)
        idx = (torch.arange(nb, device=dev).unsqueeze(1) * k + miss.to(dev)).reshape(-1)
        work.view(nb * k, L)[idx] = 0xA5
        rec_rows = torch.empty((nb, min(k, r), L), dtype=torch.uint8, device=dev)
    stream = torch.cuda.current_stream(dev)
    # The decode plan needs only the presence masks and block numbers, not the repairs: it runs on a
    # second stream beside the encode (independent work, as a receiver plans from packet headers while
    # the data streams in), and the apply waits for it.  The plan starts after the previous pass's
    # apply (it rewrites the workspace that apply reads).
    plan_stream = torch.cuda.Stream(dev) if e else None

    def step(ev=None):
        for p in range(passes):
            m = min(nb, share - p * nb)
            fb = fbn_base_of(g0 + p * nb)
            tm = ev if ev and p == 0 else None
            if e:
                go = torch.cuda.Event()
                go.record(stream)
                plan_stream.wait_event(go)
                if tm:
                    tm[4].record(plan_stream)
                eng.rlc_decode_plan(sp, rp, k, r, m, ws, fbn_base=fb, stream=plan_stream)
                if tm:
                    tm[5].record(plan_stream)
                planned = torch.cuda.Event()
                planned.record(plan_stream)
            if tm:
                tm[0].record(stream)
            eng.rlc_encode(src, rep, k, r, L, nblocks=m, fbn_base=fb)
            if tm:
                tm[1].record(stream)
            if e:
                stream.wait_event(planned)
                if tm:
                    tm[2].record(stream)
                eng.rlc_decode_apply_packed(work, rep, rec_rows, status, recovered, k, r, L, m, ws)
                if tm:
                    tm[3].record(stream)
            elif tm:
                tm[2].record(stream)
                tm[3].record(stream)

    n_rec = n_ub = 0

    def gate():
        """correctness gate on the benchmarked data: every recovered block's erased rows equal the originals"""
        nonlocal n_rec, n_ub
        ok = status == 0
        if passes == 1:
            check_recovered(torch, rec_rows, src, ok, miss, nb, k, L, "decode did not restore the sources")
        n_rec = int(ok.sum())
        n_ub = int((status == 2).sum())

    n_enc_checked = 0

    def encode_gate(samples=4096):
        """Encode-only workloads (configs[3]): the repairs of EVERY pass decode back to the sources.  Per
        pass, a sample of blocks spread over the pass (its own block numbers, fbn_base_of(g0 + p * nb) + b,
        stated here independently of the step) loses min(k, r) random sources and is decoded from its
        repairs; every block the decode recovers must equal the originals, and nearly all must recover (the
        rest are singular draws or the reference's own crash patterns, flagged per block).  The last pass is
        checked on the timed step's own repairs first; the earlier passes are re-coded untimed, by the same
        call on the same resident sources.  The line prints only after every sample matches."""
        nonlocal n_enc_checked
        em = min(k, r)
        g = torch.Generator(device="cpu").manual_seed(0xC0FFEE + rank)
        rp_s = torch.zeros((samples, 2), dtype=torch.int64, device=dev)
        rp_s[:, 0] = (1 << r) - 1 if r < 64 else -1
        for p in reversed(range(passes)):
            m = min(nb, share - p * nb)
            fb = fbn_base_of(g0 + p * nb)
            if p != passes - 1:
                eng.rlc_encode(src, rep, k, r, L, nblocks=m, fbn_base=fb)
            n = min(samples, m)
            idx = torch.randperm(m, generator=g)[:n].sort().values.to(dev)
            s_src, s_rep = src[idx], rep[idx]
            fbn = ((idx + fb) & 0xFFFFFF).to(torch.int32)
            sp_s, miss_s = make_erasures(torch, n, k, em, 0x5A17 + p, dev)
            w = s_src.clone()
            rows = (torch.arange(n, device=dev).unsqueeze(1) * k + miss_s.to(dev)).reshape(-1)
            w.view(n * k, L)[rows] = 0
            st = torch.empty(n, dtype=torch.uint8, device=dev)
            rec = torch.empty((n, 2), dtype=torch.int64, device=dev)
            eng.rlc_decode(w, s_rep, sp_s, rp_s[:n], st, rec, k, r, L, nblocks=n, fbn=fbn)
            torch.cuda.synchronize()
            ok = st == 0
            assert int(ok.sum()) >= 0.9 * n, f"encode gate, pass {p}: only {int(ok.sum())} of {n} sampled blocks decode"
            assert bool((w[ok] == s_src[ok]).all()), f"encode gate, pass {p}: decoded sources differ from the originals"
            n_enc_checked += int(ok.sum())

    for _ in range(args.warmup):
        step()
    # the gate reads the last timed step's outputs, after the timed region: run between the warmup and
    # the timed steps, its host-side seconds let the GPU idle and the timed steps start cold
    gate_first = os.environ.get("PQUIC_BENCH_GATE_FIRST") == "1"  # A/B of the older order
    torch.cuda.synchronize()
    if e and gate_first:
        gate()

    evs = [[torch.cuda.Event(enable_timing=True) for _ in range(6)] for _ in range(args.steps)]
    if dist:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for s_ in range(args.steps):
        step(evs[s_])
    torch.cuda.synchronize()
    t_rank = time.perf_counter() - t0
    if dist:
        dist.barrier()
    t1 = time.perf_counter()
    elapsed = t1 - t0
    if e and not gate_first and args.steps + args.warmup > 0:
        gate()
    if not e and args.steps + args.warmup > 0:
        encode_gate()
    # first pass of a step: encode, apply (includes the zero/undetermined rule), plan (its own stream)
    enc_ms, apply_ms = (sum(ev[i].elapsed_time(ev[i + 1]) for ev in evs) / args.steps for i in (0, 2))
    plan_ms = sum(ev[4].elapsed_time(ev[5]) for ev in evs) / args.steps if e else 0.0
    dec_ms = plan_ms + apply_ms
    per_rank = rank_devices = None
    if dist:
        t = torch.tensor([elapsed], dtype=torch.float64, device=dev if backend == "nccl" else "cpu")
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
        tr = torch.tensor([t_rank], dtype=torch.float64, device=dev if backend == "nccl" else "cpu")
        allr = [torch.zeros_like(tr) for _ in range(world)]
        dist.all_gather(allr, tr)
        per_rank = [round(float(x.item()) / args.steps * 1e3, 3) for x in allr]
        dv = torch.tensor([float(local)], dtype=torch.float64, device=dev if backend == "nccl" else "cpu")
        alld = [torch.zeros_like(dv) for _ in range(world)]
        dist.all_gather(alld, dv)
        rank_devices = [int(x.item()) for x in alld]

    total_blocks = world * share if cfg["scaling"] == "weak" else cfg["total"]
    value = total_blocks * k * L * args.steps / elapsed / 2**30
    payload = nb * k * L  # resident blocks (one pass)
    enc_bytes = (k + r) * L * nb                 # read k sources, write r repairs per block
    app_bytes = (k + e) * L * n_rec              # read k received symbols, write e per recovered block
    enc_gbs = enc_bytes / (enc_ms * 1e-3) / 1e9
    app_gbs = app_bytes / (apply_ms * 1e-3) / 1e9 if e else 0.0
    tag = f"k{k}_r{r}" + ("" if L == 1200 else f"_L{L}")
    enc_kernel = encode_kernel_name(k, r, L)
    legs = {
        f"rlc_encode_{tag}": {"kernel": enc_kernel, "ms": round(enc_ms, 3), "blocks": nb,
                              "payload_GiB_s": round(payload / (enc_ms * 1e-3) / 2**30, 2),
                              "algorithmic_GB_s": round(enc_gbs, 1), "hbm_frac": round(enc_gbs / HBM_PEAK_GBS, 4),
                              "bytes_per_launch": enc_bytes, "traffic": load_traffic(f"rlc_encode_{tag}", nb)},
    }
    if e:
        legs[f"rlc_decode_k{k}_e{e}"] = {
            "ms": round(dec_ms, 3), "plan_ms": round(plan_ms, 3), "apply_ms": round(apply_ms, 3),
            "plan_stream": "second stream, beside the encode (needs only masks and block numbers)",
            "payload_GiB_s": round(payload / (dec_ms * 1e-3) / 2**30, 2),
            "apply_kernel": apply_kernel_name(k, r, L), "apply_algorithmic_GB_s": round(app_gbs, 1),
            "apply_hbm_frac": round(app_gbs / HBM_PEAK_GBS, 4), "recovered_blocks": n_rec,
            "ref_ub_blocks": n_ub, "traffic": load_traffic(f"rlc_decode_apply_k{k}_e{e}", nb)}
    if e:
        del work, ws, rec_rows
    default = args.config == "k16" and (k, r, e, L) == (16, 4, 4, 1200)
    if default and not args.no_legs and world == 1:
        # §8f row 2: the repair symbols of the whole batch as FEC frames (header + payload) on the device
        fstride = (14 + L + 15) // 16 * 16
        frames = torch.empty(nb * r * fstride, dtype=torch.uint8, device=dev)
        fbn_base = fbn_base_of(g0)
        eng.write_repair_frames(rep, frames, nb, r, L, L, fstride, k, r, fbn_base=fbn_base)
        a, b_ = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record(stream)
        for _ in range(5):
            eng.write_repair_frames(rep, frames, nb, r, L, L, fstride, k, r, fbn_base=fbn_base)
        b_.record(stream)
        torch.cuda.synchronize()
        ms = a.elapsed_time(b_) / 5
        fb = nb * r * (L + fstride)  # read the repairs, write the frame slots
        legs["repair_frames_k16_r4"] = {"kernel": "k_write_repair_frames16", "frames": nb * r, "frame_stride": fstride,
                                        "ms": round(ms, 3), "algorithmic_GB_s": round(fb / (ms * 1e-3) / 1e9, 1)}
        del frames
    if default and not args.no_legs and world == 1:
        # north-star leg: k = 32, r = 8 encode, 2^21 blocks (one GPU's share of config 4)
        nb2, k2, r2 = 1 << 21, 32, 8
        del src, rep
        torch.cuda.empty_cache()
        s2 = torch.empty((nb2, k2, L), dtype=torch.uint8, device=dev)
        eng.synth_fill(s2, s2.numel(), 0x5EEDF3C0, 0)
        r2t = torch.empty((nb2, r2, L), dtype=torch.uint8, device=dev)
        for _ in range(2):
            eng.rlc_encode(s2, r2t, k2, r2, L)
        a, b_ = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record(stream)
        for _ in range(5):
            eng.rlc_encode(s2, r2t, k2, r2, L)
        b_.record(stream)
        torch.cuda.synchronize()
        ms = a.elapsed_time(b_) / 5
        gbs = (k2 + r2) * L * nb2 / (ms * 1e-3) / 1e9
        legs["rlc_encode_k32_r8"] = {"kernel": "k_rlc_encode_bs<8,16>", "ms": round(ms, 3), "blocks": nb2,
                                     "payload_GiB_s": round(nb2 * k2 * L / (ms * 1e-3) / 2**30, 2),
                                     "algorithmic_GB_s": round(gbs, 1), "hbm_frac": round(gbs / HBM_PEAK_GBS, 4),
                                     "traffic": load_traffic("rlc_encode_k32_r8", nb2)}
        # §8f row 3, the window framework every shipped RLC manifest uses: window blocks carry block
        # number 0, so all windows share their coefficients; overlapping windows run on
        # k_rlc_encode_sc (2 KiB chunks of the windows x bytes space per case), windows that do not
        # overlap on the block kernel.  Windows of 32 advancing by 8 (each source in 4 windows) and
        # adjacent windows (the same bytes as the k32 r8 block leg).
        sym = s2.view(-1, L)
        for wname, wstep in (("adjacent", 32), ("step8", 8)):
            nw = nb2
            for _ in range(2):
                eng.rlc_window_encode(sym, r2t, nw, wstep, k2, r2, L)
            a.record(stream)
            for _ in range(5):
                eng.rlc_window_encode(sym, r2t, nw, wstep, k2, r2, L)
            b_.record(stream)
            torch.cuda.synchronize()
            wms = a.elapsed_time(b_) / 5
            # bytes a pass must move at least: every source row once, every repair once
            min_bytes = ((nw - 1) * wstep + k2 + nw * r2) * L
            wgbs = min_bytes / (wms * 1e-3) / 1e9
            legs[f"rlc_window_encode_k32_r8_{wname}"] = {
                "kernel": "k_rlc_encode_sc<8>" if wstep < k2 else "k_rlc_encode_bs<8,16>", "ms": round(wms, 3),
                "windows": nw, "step": wstep,
                "window_payload_GiB_s": round(nw * k2 * L / (wms * 1e-3) / 2**30, 2),
                "min_bytes_GB_s": round(wgbs, 1), "hbm_frac": round(wgbs / HBM_PEAK_GBS, 4)}
        del s2, r2t, sym
        torch.cuda.empty_cache()
        # configs[4]: jumbo 9000-B symbols, k = 64 r = 16, encode + decode of 16 erasures
        legs["rlc_k64_r16_L9000"] = rlc_leg(torch, eng, dev, 64, 16, 9000, 1 << 16, 16)
        # configs[0]'s XOR scheme (k = 4, r = 1) at GPU scale: encode + single-erasure recover
        legs["xor_k4_r1"] = xor_leg(torch, eng, dev, 4, L, 1 << 22)
    if default and not args.no_legs and not args.no_pcie and world == 1:
        # the host-path legs last, once the device legs have freed their tensors (they use buffers of their
        # own: page-locked rows, registered arenas); the batching and hook legs in a process of their own
        torch.cuda.empty_cache()
        legs.update(pcie_legs(torch, args, dev))
        legs.update(host_legs_child(args, dev.index or 0))

    if rank == 0:
        if not e or enc_ms >= apply_ms:
            roof = {"bound": "hbm", "kernel": f"{enc_kernel} (RLC encode k={k} r={r})",
                    "achieved": round(enc_gbs, 1), "bytes_per_launch": enc_bytes, "launch_ms": round(enc_ms, 4),
                    "traffic": load_traffic(f"rlc_encode_{tag}", nb)}
        else:
            roof = {"bound": "hbm", "kernel": f"{apply_kernel_name(k, r, L)} (RLC decode apply k={k} e={e})",
                    "achieved": round(app_gbs, 1), "bytes_per_launch": app_bytes, "launch_ms": round(apply_ms, 4),
                    "traffic": load_traffic(f"rlc_decode_apply_k{k}_e{e}", nb)}
        # the PMC traffic figure is measured in its own rocprofv3 --pmc passes, not in this run: name its build
        roof["traffic_measured_at"] = traffic_build(f"rlc_encode_{tag}" if (not e or enc_ms >= apply_ms)
                                                    else f"rlc_decode_apply_k{k}_e{e}")
        roof.update({"peak": HBM_PEAK_GBS, "unit": "GB/s", "frac": round(roof["achieved"] / HBM_PEAK_GBS, 4),
                     "measured_copy_peak": MEASURED_COPY_GBS,
                     "frac_of_measured_copy": round(roof["achieved"] / MEASURED_COPY_GBS, 4),
                     "measured_mix41_peak": MEASURED_MIX41_GBS})
        if args.config == "k16":
            roof.update({"pattern_ceiling": PATTERN_CEILING_GBS,
                         "frac_of_pattern_ceiling": round(roof["achieved"] / PATTERN_CEILING_GBS, 4)})
        conf = {"workload": cfg["workload"], "k": k, "r": r, "erasures": e, "symbol_bytes": L,
                "blocks_per_gpu": share, "blocks_total": total_blocks, "resident_blocks_per_gpu": nb,
                "passes_per_step": passes,
                "parallelism": f"independent FEC blocks, {world} GPU(s), no collective"}
        if e:
            conf["decode_output"] = ("recovered symbols into new rows, packed per block (as fec_recover "
                                     "allocates each recovered symbol anew)")
        if not e:
            conf["encode_gate"] = {"passes_checked": passes, "blocks_decoded_back": n_enc_checked,
                                   "method": "per pass, sampled blocks lose min(k, r) sources and decode back "
                                             "from the pass's repairs at independently stated block numbers"}
        if passes > 1:
            conf["note"] = (f"a GPU's share ({share} blocks) exceeds HBM: each step codes it in {passes} passes "
                            f"over {nb} resident blocks, block numbers advancing per pass")
        out = {"metric": METRIC, "value": round(value, 3), "unit": "GiB/s", "n_gpus": world,
               "steps": args.steps, "warmup": args.warmup,
               "ms_per_step": round(elapsed / args.steps * 1e3, 3), "higher_is_better": True,
               "scaling": cfg["scaling"], "vs_baseline": None, "dtype": "u8", "data": "synthetic",
               "config": conf, "roofline": roof, "cpu_baseline": cpu, "legs": legs}
        if per_rank:
            out["per_rank_ms_per_step"] = per_rank
            out["per_rank_device"] = rank_devices
            out["launcher"] = "bench.py child processes" if os.environ.get("PQUIC_BENCH_LAUNCHED") else "torchrun"
        print(json.dumps(out))
    if dist:
        dist.barrier()
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
