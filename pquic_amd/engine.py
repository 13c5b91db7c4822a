"""ctypes mirror of include/fecgpu.h (batched device-resident FEC engine).

Buffers are torch CUDA tensors (HBM allocations) or raw device addresses; kernels run on
the given HIP stream (default: torch's current stream), so torch.cuda.Event timing
brackets exactly the engine's launches.
"""
from __future__ import annotations

import ctypes as C
import os

PKG = os.path.dirname(os.path.abspath(__file__))
# PQUIC_AMD_LIB selects another in-tree build of the same library (A/B experiments, tools/)
LIB_PATH = os.environ.get("PQUIC_AMD_LIB") or os.path.join(PKG, "lib", "libpquic_fec.so")

OK, ERR_INVALID, ERR_HIP, ERR_NO_DEVICE, ERR_NOMEM = 0, -1, -2, -3, -4
BLOCK_RECOVERED, BLOCK_NOTHING, BLOCK_REF_UB = 0, 1, 2

_lib = None


class FecGpuError(RuntimeError):
    pass


class FecGpuStats(C.Structure):
    _fields_ = [("encode_calls", C.c_uint64), ("encode_blocks", C.c_uint64),
                ("decode_calls", C.c_uint64), ("decode_blocks", C.c_uint64),
                ("pinned_registry_hits", C.c_uint64), ("pinned_registry_misses", C.c_uint64),
                ("yield_slices", C.c_uint64), ("yield_waits", C.c_uint64)]


def load_library(path: str = LIB_PATH, private: bool = False):
    """Load libpquic_fec.so.  Raises if it is missing -- never falls back to CPU.
    private=True loads another build side by side (its own handle; in-process A/B tools)."""
    global _lib
    if _lib is not None and not private:
        return _lib
    if not os.path.exists(path):
        raise FecGpuError(f"{path} not built: run `python -c 'import __graft_entry__ as g; g.build()'`")
    L = C.CDLL(path)
    v, u64, u32, sz = C.c_void_p, C.c_uint64, C.c_uint32, C.c_size_t
    L.fecgpu_init.argtypes = [C.c_int]
    L.fecgpu_version.restype = C.c_char_p
    L.fecgpu_last_error.restype = C.c_char_p
    L.fecgpu_rlc_encode.argtypes = [v, v, u64, u32, u32, u32, u32, v, v]
    L.fecgpu_xor_encode.argtypes = [v, v, u64, u32, u32, v]
    L.fecgpu_rlc_window_encode.argtypes = [v, u64, u32, u32, u32, u32, v, v]
    L.fecgpu_write_repair_frames.argtypes = [v, u64, u32, u32, C.c_uint16, u32, v, C.c_uint8, C.c_uint8, v, u32, v]
    L.fecgpu_rlc_decode_workspace.argtypes = [u64, u32, u32]
    L.fecgpu_rlc_decode_workspace.restype = sz
    L.fecgpu_rlc_decode.argtypes = [v, v, u64, u32, u32, u32, u32, v, v, v, v, v, v, sz, v]
    L.fecgpu_xor_decode.argtypes = [v, v, u64, u32, u32, v, v, v, v, v]
    if hasattr(L, "fecgpu_xor_decode_to") or not private:  # a private (A/B) load may be an older build
        L.fecgpu_xor_decode_to.argtypes = [v, v, v, u64, u32, u32, v, v, v, v, v]
    L.fecgpu_rlc_decode_plan.argtypes = [u64, u32, u32, u32, v, v, v, v, sz, v]
    L.fecgpu_rlc_decode_plan_seeded.argtypes = [u64, u32, u32, v, v, v, v, sz, v]
    L.fecgpu_rlc_decode_seeded.argtypes = [v, v, u64, u32, u32, u32, v, v, v, v, v, v, sz, v]
    L.fecgpu_rlc_decode_apply.argtypes = [v, v, u64, u32, u32, u32, v, v, v, sz, v]
    L.fecgpu_rlc_decode_apply_to.argtypes = [v, v, v, u64, u32, u32, u32, v, v, v, sz, v]
    if private and not hasattr(L, "fecgpu_rlc_decode_apply_packed"):  # an older build (A/B baselines)
        pass
    else:
        L.fecgpu_rlc_decode_apply_packed.argtypes = [v, v, v, u64, u32, u32, u32, v, v, v, sz, v]
    L.fecgpu_synth_fill.argtypes = [v, u64, u64, u64, v]
    L.fecgpu_get_stats.argtypes = [C.POINTER(FecGpuStats)]
    L.fecgpu_set_knob.argtypes = [C.c_char_p, C.c_int]
    L.fecgpu_get_knob.argtypes = [C.c_char_p, C.POINTER(C.c_int)]
    L.fecgpu_host_ctx_create.argtypes = [C.c_int, C.c_int, sz]
    L.fecgpu_host_ctx_create.restype = v
    L.fecgpu_host_ctx_destroy.argtypes = [v]
    L.fecgpu_rlc_encode_host.argtypes = [v, v, v, u64, u32, u32, u32, u32, v]
    L.fecgpu_rlc_decode_host.argtypes = [v, v, v, u64, u32, u32, u32, u32, v, v, v, v, v]
    L.fecgpu_rlc_decode_host_seeded.argtypes = [v, v, v, u64, u32, u32, u32, v, v, v, v, v]
    L.fecgpu_xor_encode_host.argtypes = [v, v, v, u64, u32, u32]
    L.fecgpu_xor_decode_host.argtypes = [v, v, v, u64, u32, u32, v, v, v, v]
    L.fecgpu_host_register.argtypes = [v, sz]
    L.fecgpu_host_unregister.argtypes = [v]
    L.fecgpu_host_device_address.argtypes = [v, sz, C.POINTER(u64)]
    L.fecgpu_block_svc_create.argtypes = [C.c_int]
    L.fecgpu_block_svc_create.restype = v
    L.fecgpu_block_svc_destroy.argtypes = [v]
    L.fecgpu_block_svc_rlc_encode.argtypes = [v, v, v, u32, u32, u32, u32]
    L.fecgpu_block_svc_rlc_decode_seeded.argtypes = [v, v, v, v, u32, u32, u32, v, v, v, v, v]
    L.fecgpu_block_svc_launches.argtypes = [v]
    L.fecgpu_block_svc_launches.restype = u64
    if hasattr(L, "fecgpu_block_svc_set_deadline"):  # older builds (A/B baselines) lack these
        L.fecgpu_block_svc_set_deadline.argtypes = [v, u64]
        L.fecgpu_block_svc_deadline_misses.argtypes = [v]
        L.fecgpu_block_svc_deadline_misses.restype = u64
    if hasattr(L, "fecgpu_block_svc_last_stamps"):
        L.fecgpu_block_svc_last_stamps.argtypes = [v, C.POINTER(u64)]
    if hasattr(L, "fecgpu_block_svc_worker_running"):
        L.fecgpu_block_svc_worker_running.argtypes = [v]
    if hasattr(L, "fecgpu_rlc_decode_rows"):
        L.fecgpu_rlc_decode_rows.argtypes = [v, v, u64, u32, u32, u32, v, v, v, v, v, v, sz, v]
        L.fecgpu_rlc_decode_rows_host.argtypes = [v, v, v, u64, u32, u32, u32, v, v, v, v, v]
    if not private:
        _lib = L
    return L


def _addr(x):
    if x is None:
        return None
    if isinstance(x, int):
        return x
    if hasattr(x, "data_ptr"):
        return x.data_ptr()
    return x.ctypes.data  # numpy (host-resident path)


class Engine:
    """Batched FEC engine on one device.  Mirrors fecgpu_* one to one."""

    def __init__(self, device: int = 0, lib_path: str | None = None):
        import torch
        self.torch = torch
        self.lib = load_library(lib_path, private=True) if lib_path else load_library()
        self.device = device
        rc = self.lib.fecgpu_init(device)
        if rc != OK:
            raise FecGpuError(f"fecgpu_init({device}) = {rc}: {self.err()}")

    # ------------------------------------------------------------------ helpers
    def err(self) -> str:
        return self.lib.fecgpu_last_error().decode()

    def version(self) -> str:
        return self.lib.fecgpu_version().decode()

    def _stream(self, stream):
        if stream is None:
            stream = self.torch.cuda.current_stream(self.device)
        return C.c_void_p(stream.cuda_stream if hasattr(stream, "cuda_stream") else int(stream))

    def _check(self, rc, what):
        if rc != OK:
            raise FecGpuError(f"{what} failed ({rc}): {self.err()}")

    def get_knob(self, name: str) -> int:
        v = C.c_int(0)
        self._check(self.lib.fecgpu_get_knob(name.encode(), C.byref(v)), f"fecgpu_get_knob({name})")
        return v.value

    def set_knob(self, name: str, value: int):
        self._check(self.lib.fecgpu_set_knob(name.encode(), int(value)), f"fecgpu_set_knob({name})")

    def knob(self, name: str, value: int):
        """Context manager: an experiment knob (fecgpu_set_knob) set for the duration of a block."""
        import contextlib

        @contextlib.contextmanager
        def cm():
            old = self.get_knob(name)
            self.set_knob(name, value)
            try:
                yield
            finally:
                self.set_knob(name, old)
        return cm()

    def stats(self) -> dict:
        s = FecGpuStats()
        self.lib.fecgpu_get_stats(C.byref(s))
        return {f: getattr(s, f) for f, _ in s._fields_}

    # ------------------------------------------------------------------ encode
    def rlc_encode(self, src, rep, k: int, r: int, L: int, nblocks: int | None = None,
                   fbn_base: int = 0, fbn=None, stream=None):
        nb = nblocks if nblocks is not None else src.numel() // (k * L)
        self._check(self.lib.fecgpu_rlc_encode(_addr(src), _addr(rep), nb, k, r, L, fbn_base,
                                               _addr(fbn), self._stream(stream)), "fecgpu_rlc_encode")
        return rep

    def rlc_window_encode(self, symbols, rep, nwindows: int, step: int, k: int, r: int, L: int, stream=None):
        """Sliding-window encode: window w = symbols[w*step : w*step + k], block number 0."""
        self._check(self.lib.fecgpu_rlc_window_encode(_addr(symbols), nwindows, step, k, r, L, _addr(rep),
                                                      self._stream(stream)), "fecgpu_rlc_window_encode")
        return rep

    def write_repair_frames(self, rep, frames, nblocks: int, r: int, L: int, data_length: int, frame_stride: int,
                            nss: int, nrs: int, fbn_base: int = 0, fbn=None, stream=None):
        """FEC frames (header + payload) for every repair of a batch, on the device."""
        self._check(self.lib.fecgpu_write_repair_frames(_addr(rep), nblocks, r, L, data_length, fbn_base, _addr(fbn),
                                                        nss, nrs, _addr(frames), frame_stride, self._stream(stream)),
                    "fecgpu_write_repair_frames")
        return frames

    def xor_encode(self, src, rep, k: int, L: int, nblocks: int | None = None, stream=None):
        nb = nblocks if nblocks is not None else src.numel() // (k * L)
        self._check(self.lib.fecgpu_xor_encode(_addr(src), _addr(rep), nb, k, L, self._stream(stream)),
                    "fecgpu_xor_encode")
        return rep

    # ------------------------------------------------------------------ decode
    def decode_workspace_bytes(self, nblocks: int, k: int, r: int) -> int:
        return int(self.lib.fecgpu_rlc_decode_workspace(nblocks, k, r))

    def alloc_workspace(self, nblocks: int, k: int, r: int):
        n = self.decode_workspace_bytes(nblocks, k, r)
        return self.torch.empty(max(n, 16), dtype=self.torch.uint8, device=f"cuda:{self.device}")

    def rlc_decode(self, src, rep, src_present, rep_present, status, recovered, k: int, r: int,
                   L: int, nblocks: int | None = None, fbn_base: int = 0, fbn=None,
                   workspace=None, stream=None):
        nb = nblocks if nblocks is not None else src.numel() // (k * L)
        if workspace is None:
            workspace = self.alloc_workspace(nb, k, r)
        self._check(self.lib.fecgpu_rlc_decode(
            _addr(src), _addr(rep), nb, k, r, L, fbn_base, _addr(fbn), _addr(src_present),
            _addr(rep_present), _addr(status), _addr(recovered), _addr(workspace),
            workspace.numel(), self._stream(stream)), "fecgpu_rlc_decode")
        return status, recovered

    def rlc_decode_seeded(self, src, rep, rep_seed, src_present, rep_present, status, recovered, k: int, r: int,
                          L: int, nblocks: int | None = None, workspace=None, stream=None):
        """fecgpu_rlc_decode_seeded: every received repair's coefficients seeded by its own FPID,
        rep_seed[b * r + i] (u32 device array) -- the sliding-window framework's blocks."""
        nb = nblocks if nblocks is not None else src.numel() // (k * L)
        if workspace is None:
            workspace = self.alloc_workspace(nb, k, r)
        self._check(self.lib.fecgpu_rlc_decode_seeded(
            _addr(src), _addr(rep), nb, k, r, L, _addr(rep_seed), _addr(src_present), _addr(rep_present),
            _addr(status), _addr(recovered), _addr(workspace), workspace.numel(), self._stream(stream)),
            "fecgpu_rlc_decode_seeded")
        return status, recovered

    def rlc_decode_stages(self, src, rep, src_present, rep_present, status, recovered, k, r, L, nblocks,
                          workspace, fbn_base=0, stream=None, events=None, dst=None, packed=False):
        """fecgpu_rlc_decode as its two stages (plan, apply); events[i] (if given) recorded before
        stage i and events[2] after the last, on the launch stream.  dst: write the recovered rows
        there (src's layout, fecgpu_rlc_decode_apply_to; packed=True: [nblocks][min(k, r)] rows,
        fecgpu_rlc_decode_apply_packed) instead of into src."""
        st = self._stream(stream)
        torch_stream = stream if stream is not None else self.torch.cuda.current_stream(self.device)
        rec = (lambda i: events[i].record(torch_stream)) if events else (lambda i: None)
        rec(0)
        self._check(self.lib.fecgpu_rlc_decode_plan(nblocks, k, r, fbn_base, None, _addr(src_present),
                                                    _addr(rep_present), _addr(workspace), workspace.numel(), st),
                    "fecgpu_rlc_decode_plan")
        rec(1)
        if dst is not None and packed:
            self._check(self.lib.fecgpu_rlc_decode_apply_packed(_addr(src), _addr(rep), _addr(dst), nblocks, k, r,
                                                                L, _addr(status), _addr(recovered),
                                                                _addr(workspace), workspace.numel(), st),
                        "fecgpu_rlc_decode_apply_packed")
        elif dst is None:
            self._check(self.lib.fecgpu_rlc_decode_apply(_addr(src), _addr(rep), nblocks, k, r, L, _addr(status),
                                                         _addr(recovered), _addr(workspace), workspace.numel(), st),
                        "fecgpu_rlc_decode_apply")
        else:
            self._check(self.lib.fecgpu_rlc_decode_apply_to(_addr(src), _addr(rep), _addr(dst), nblocks, k, r, L,
                                                            _addr(status), _addr(recovered), _addr(workspace),
                                                            workspace.numel(), st), "fecgpu_rlc_decode_apply_to")
        rec(2)
        return status, recovered

    def rlc_decode_plan(self, src_present, rep_present, k, r, nblocks, workspace, fbn_base=0, fbn=None,
                        stream=None):
        """fecgpu_rlc_decode_plan: coefficient-only stage (needs only the presence masks)."""
        self._check(self.lib.fecgpu_rlc_decode_plan(nblocks, k, r, fbn_base, _addr(fbn), _addr(src_present),
                                                    _addr(rep_present), _addr(workspace), workspace.numel(),
                                                    self._stream(stream)), "fecgpu_rlc_decode_plan")

    def rlc_decode_apply(self, src, rep, status, recovered, k, r, L, nblocks, workspace, stream=None):
        """fecgpu_rlc_decode_apply: the data pass plus the zero/undetermined rule."""
        self._check(self.lib.fecgpu_rlc_decode_apply(_addr(src), _addr(rep), nblocks, k, r, L, _addr(status),
                                                     _addr(recovered), _addr(workspace), workspace.numel(),
                                                     self._stream(stream)), "fecgpu_rlc_decode_apply")
        return status, recovered

    def rlc_decode_apply_to(self, src, rep, dst, status, recovered, k, r, L, nblocks, workspace, stream=None):
        """fecgpu_rlc_decode_apply_to: as apply, recovered symbols written to dst (src's layout)."""
        self._check(self.lib.fecgpu_rlc_decode_apply_to(_addr(src), _addr(rep), _addr(dst), nblocks, k, r, L,
                                                        _addr(status), _addr(recovered), _addr(workspace),
                                                        workspace.numel(), self._stream(stream)),
                    "fecgpu_rlc_decode_apply_to")
        return status, recovered

    def rlc_decode_apply_packed(self, src, rep, dst, status, recovered, k, r, L, nblocks, workspace, stream=None):
        """fecgpu_rlc_decode_apply_packed: as apply, recovered symbols packed into dst [nblocks][min(k, r)][L]
        (row u = the u-th missing source of the block, ascending)."""
        self._check(self.lib.fecgpu_rlc_decode_apply_packed(_addr(src), _addr(rep), _addr(dst), nblocks, k, r, L,
                                                            _addr(status), _addr(recovered), _addr(workspace),
                                                            workspace.numel(), self._stream(stream)),
                    "fecgpu_rlc_decode_apply_packed")
        return status, recovered

    def xor_decode(self, src, rep, src_present, rep_present, status, recovered, k: int, L: int,
                   nblocks: int | None = None, stream=None):
        nb = nblocks if nblocks is not None else src.numel() // (k * L)
        self._check(self.lib.fecgpu_xor_decode(_addr(src), _addr(rep), nb, k, L, _addr(src_present),
                                               _addr(rep_present), _addr(status), _addr(recovered),
                                               self._stream(stream)), "fecgpu_xor_decode")
        return status, recovered

    def xor_decode_to(self, src, rep, dst, src_present, rep_present, status, recovered, k: int, L: int,
                      nblocks: int | None = None, stream=None):
        """fecgpu_xor_decode_to: the recovered symbol of block b into dst[b] (one row per block); src is read only."""
        nb = nblocks if nblocks is not None else src.numel() // (k * L)
        self._check(self.lib.fecgpu_xor_decode_to(_addr(src), _addr(rep), _addr(dst), nb, k, L, _addr(src_present),
                                                  _addr(rep_present), _addr(status), _addr(recovered),
                                                  self._stream(stream)), "fecgpu_xor_decode_to")
        return status, recovered

    def synth_fill(self, dst, nbytes: int, seed: int, offset: int = 0, stream=None):
        self._check(self.lib.fecgpu_synth_fill(_addr(dst), nbytes, seed, offset, self._stream(stream)),
                    "fecgpu_synth_fill")
        return dst


class HostPath:
    """Host-resident entry points (include/fecgpu.h 'Host-resident path'): host buffers in,
    host buffers out, H2D/D2H overlapped with the kernels on `nstreams` streams."""

    def __init__(self, device: int = 0, nstreams: int = 3, chunk_bytes: int = 64 << 20):
        self.lib = load_library()
        self.ctx = self.lib.fecgpu_host_ctx_create(device, nstreams, chunk_bytes)
        if not self.ctx:
            raise FecGpuError(f"fecgpu_host_ctx_create({device}) failed: {self.lib.fecgpu_last_error().decode()}")

    def close(self):
        if self.ctx:
            self.lib.fecgpu_host_ctx_destroy(self.ctx)
            self.ctx = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def _chk(self, rc, what):
        if rc != OK:
            raise FecGpuError(f"{what} failed ({rc}): {self.lib.fecgpu_last_error().decode()}")

    def rlc_encode(self, src, rep, nblocks, k, r, L, fbn_base=0):
        self._chk(self.lib.fecgpu_rlc_encode_host(self.ctx, _addr(src), _addr(rep), nblocks, k, r, L, fbn_base,
                                                  None), "fecgpu_rlc_encode_host")

    def rlc_decode(self, src, rep, sp, rp, status, rec, nblocks, k, r, L, fbn_base=0):
        self._chk(self.lib.fecgpu_rlc_decode_host(self.ctx, _addr(src), _addr(rep), nblocks, k, r, L, fbn_base,
                                                  None, _addr(sp), _addr(rp), _addr(status), _addr(rec)),
                  "fecgpu_rlc_decode_host")

    def rlc_decode_seeded(self, src, rep, seeds, sp, rp, status, rec, nblocks, k, r, L):
        self._chk(self.lib.fecgpu_rlc_decode_host_seeded(self.ctx, _addr(src), _addr(rep), nblocks, k, r, L,
                                                         _addr(seeds), _addr(sp), _addr(rp), _addr(status),
                                                         _addr(rec)), "fecgpu_rlc_decode_host_seeded")
