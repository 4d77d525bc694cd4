"""Python surface of the MI355X decoder, mirroring the reference's decode boundary.

* ``decode_bits(llrs, H, bp_iterations, batch_size, clamp_value)`` — drop-in for
  ``pytorch/ofdm/ofdm_functions.py:131-163`` (same arguments, float64 0/1 output, rows past
  ``(N // batch_size) * batch_size`` left 0, tanh sum-product, fp32 arithmetic).
* ``decoder`` — alias for the same function: the reference's stale scripts call a missing
  ``decoder(...)`` with these 5 arguments (``evaluate.py:9,117``).
* ``BeliefPropagation(H, iterations)`` — ``torch.nn.Module`` with ``forward(x, llr, clamp_value) -> p1`` and
  ``layer_size()``, as ``pytorch/bp/bp.py:19-62`` (used directly by ``ber_test.py:87``).
* ``decode(H, llr, max_iters, ...)`` — the general entry point (algorithms, precision, early stop,
  device tensors without host copies).

All arithmetic runs in libldpc_hip.so on the GPU; nothing here computes a message.
"""
from __future__ import annotations

import ctypes
import hashlib
import os
import threading

import numpy as np

from . import _abi
from ._abi import Params, check
from .codes import Graph, SparseCode

_ALGOS = {"tanh": _abi.ALGO_TANH_SP, "sp": _abi.ALGO_TANH_SP, "tanh_sp": _abi.ALGO_TANH_SP,
          "minsum": _abi.ALGO_MIN_SUM, "min_sum": _abi.ALGO_MIN_SUM, "ms": _abi.ALGO_MIN_SUM,
          "qminsum": _abi.ALGO_QMIN_SUM, "qms": _abi.ALGO_QMIN_SUM}


def _torch():
    import torch
    return torch


class Decoder:
    """One Tanner graph resident on one GPU (a ``ldpc_graph`` handle)."""

    def __init__(self, H, device: int = 0):
        self.lib = _abi.load()
        g = Graph.from_H(H if isinstance(H, (SparseCode, Graph)) else np.asarray(H)) if not isinstance(H, Graph) else H
        self.m, self.n, self.E = g.m, g.n, g.E
        self.device = int(device)
        h = ctypes.c_void_p()
        rp = np.ascontiguousarray(g.row_ptr, np.int32)
        ci = np.ascontiguousarray(g.col_idx, np.int32)
        check(self.lib.ldpc_graph_create(g.m, g.n, g.E, rp.ctypes.data, ci.ctypes.data, self.device, ctypes.byref(h)))
        self._h = h
        z = ctypes.c_int32()
        check(self.lib.ldpc_graph_info(self._h, None, None, None, ctypes.byref(z)))
        self.qc_z = int(z.value)
        w, f = ctypes.c_int64(), ctypes.c_int64()
        check(self.lib.ldpc_weights_layout(self._h, ctypes.byref(w), ctypes.byref(f)))
        self.weights_per_iter = int(w.value)   # compact VN weights per iteration (sum_v d_v^2)
        self.graph = g

    def __del__(self):
        h = getattr(self, "_h", None)
        if h is not None and h.value:
            try:
                self.lib.ldpc_graph_destroy(h)
            except Exception:
                pass
            self._h = None

    @staticmethod
    def params(iters, algo="tanh", clamp=10.0, alpha=1.0, beta=0.0, early_stop=False, precision="f32",
               soft="p1", qmax=15, app_max=127, qstep=1.0, force_generic=False, device_ptrs=False) -> Params:
        if algo not in _ALGOS:
            raise ValueError(f"algo must be one of {sorted(_ALGOS)}")
        if precision not in ("f32", "f64"):
            raise ValueError("precision must be 'f32' or 'f64'")
        flags = 0
        flags |= _abi.F_EARLY_STOP if early_stop else 0
        flags |= _abi.F_F64 if precision == "f64" else 0
        flags |= _abi.F_SOFT_Z if soft == "z" else 0
        flags |= _abi.F_FORCE_GENERIC if force_generic else 0
        flags |= _abi.F_DEVICE_PTRS if device_ptrs else 0
        return Params(int(iters), _ALGOS[algo], flags, float(clamp), float(alpha), float(beta), int(qmax),
                      int(app_max), float(qstep))

    def kernel_path(self, p: Params) -> str:
        """The kernel family a decode with these params runs: "qc-z<Z>", "ira-z360" or "generic-csr"."""
        s = self.lib.ldpc_kernel_path(self._h, ctypes.byref(p))
        if s is None:
            raise _abi.LdpcError(_abi.LDPC_EINVAL, self.lib.ldpc_last_error().decode(errors="replace"))
        return s.decode()

    def workspace_bytes(self, B: int, p: Params) -> int:
        out = ctypes.c_size_t()
        check(self.lib.ldpc_workspace_size(self._h, int(B), ctypes.byref(p), ctypes.byref(out)))
        return int(out.value)

    def device_weights(self, weights, iters: int, precision="f32"):
        """Compact weights (dict vn [iters][W], llr [iters][n], fin [E], fin_llr [n]; numpy or torch; any key
        None/missing = ones) -> (BPWeights struct, device tensors kept alive).  Shapes are checked here."""
        torch = _torch()
        tdt = torch.float64 if precision == "f64" else torch.float32
        dev = torch.device("cuda", self.device)
        shapes = dict(vn=(iters, self.weights_per_iter), llr=(iters, self.n), fin=(self.E,), fin_llr=(self.n,))
        keep, ptrs = [], []
        for k in ("vn", "llr", "fin", "fin_llr"):
            a = (weights or {}).get(k)
            if a is None:
                ptrs.append(None)
                continue
            t = torch.as_tensor(a).detach().to(device=dev, dtype=tdt).contiguous()
            if tuple(t.shape) != shapes[k]:
                raise ValueError(f"weights[{k!r}] must have shape {shapes[k]}, got {tuple(t.shape)}")
            keep.append(t)
            ptrs.append(t.data_ptr())
        return _abi.BPWeights(*ptrs), keep

    def decode(self, llr, iters: int, *, algo="tanh", clamp=10.0, alpha=1.0, beta=0.0, early_stop=False,
               precision="f32", soft=None, qmax=15, app_max=127, qstep=1.0, force_generic=False, stream=None,
               want_bits=True, want_iters=False, weights=None, x0=None):
        """Decode a (B, n) batch of LLRs (log P1/P0).  numpy in -> numpy out (host staging inside the
        library); torch GPU tensor in (on this decoder's device) -> torch GPU tensors out, asynchronous on
        ``stream`` (a ``torch.cuda.Stream`` or a raw ``hipStream_t`` handle as an int; default: the current
        stream; a side stream first waits for the current one, every input it reads is kept allocated until
        it has read it, and the outputs are allocated on and ordered by the side stream) with a
        torch-allocated workspace.  Returns dict(bits, soft, iters_used).
        ``weights``: weighted BP (tanh-SP only), compact layout of ``Graph.compact_weights``.
        ``x0``: initial c2v messages (B, E) in check-order — the reference's ``x`` (``bp/bp.py:43-47``);
        torch GPU tensors only (tanh-SP, no early stop, generic kernels)."""
        is_torch = type(llr).__module__.startswith("torch")
        on_gpu = is_torch and llr.is_cuda
        fdt = np.float64 if precision == "f64" else np.float32
        if weights is not None or x0 is not None:
            force_generic = True
        if x0 is not None and not on_gpu:
            raise ValueError("x0 (initial messages) needs torch GPU tensors for llr and x0")
        p = self.params(iters, algo, clamp, alpha, beta, early_stop, precision, soft or "p1", qmax, app_max,
                        qstep, force_generic, device_ptrs=on_gpu)
        wstruct, _wkeep = (self.device_weights(weights, iters, precision) if weights is not None else (None, None))

        x0t = None

        def call(*args):
            if x0t is not None:
                return self.lib.ldpc_decode_x0(self._h, args[0], args[1], ctypes.byref(p),
                                               ctypes.byref(wstruct) if wstruct is not None else None,
                                               x0t.data_ptr(), *args[2:])
            if wstruct is None:
                return self.lib.ldpc_decode_ex(self._h, args[0], args[1], ctypes.byref(p), *args[2:])
            return self.lib.ldpc_decode_weighted(self._h, args[0], args[1], ctypes.byref(p), ctypes.byref(wstruct),
                                                 *args[2:])
        if on_gpu:
            torch = _torch()
            if llr.device.index != self.device:
                raise ValueError(f"llr is on {llr.device}, this decoder's graph is on cuda:{self.device}")
            cur = torch.cuda.current_stream(llr.device)
            ext = cur if stream is None else stream
            if isinstance(ext, int) and not isinstance(ext, bool):  # a raw hipStream_t handle
                ext = torch.cuda.ExternalStream(ext, device=llr.device)
            if not isinstance(ext, torch.cuda.Stream):
                raise TypeError("stream must be a torch.cuda.Stream, an int stream handle, or None (current stream)")
            side = ext != cur
            if side:
                ext.wait_stream(cur)        # llr (and the caller's prior work) is ordered before the decode
                # every tensor the decode reads stays allocated until the decode stream has read it: the
                # caller's llr / x0 and the weights uploaded on the current stream
                for t in [llr, x0] + list(_wkeep or []):
                    if t is not None:
                        t.record_stream(ext)
            tdt = torch.float64 if precision == "f64" else torch.float32
            # conversion, outputs and workspace all live on the decode stream: the allocator recycles them in
            # that stream's order, and results are ready once `ext` reaches this point
            with torch.cuda.stream(ext):
                x = llr.detach().to(tdt).contiguous()
                if x.dim() != 2 or x.shape[1] != self.n:
                    raise RuntimeError(f"llr must be (B, {self.n}), got {tuple(x.shape)}")
                B = x.shape[0]
                dev = x.device
                if x0 is not None:
                    if x0.device != llr.device:
                        raise ValueError(f"x0 is on {x0.device}, llr on {llr.device}")
                    x0t = x0.detach().to(tdt).contiguous()
                    if tuple(x0t.shape) != (B, self.E):
                        raise RuntimeError(f"x0 must be (B, E) = ({B}, {self.E}), got {tuple(x0t.shape)}")
                bits = torch.empty((B, self.n), dtype=torch.uint8, device=dev) if want_bits else None
                sft = torch.empty((B, self.n), dtype=tdt, device=dev) if soft else None
                used = torch.empty((B,), dtype=torch.int32, device=dev) if want_iters else None
                wsb = self.workspace_bytes(B, p)
                ws = torch.empty((max(wsb, 1),), dtype=torch.uint8, device=dev)
                check(call(x.data_ptr(), B, bits.data_ptr() if bits is not None else None,
                           sft.data_ptr() if sft is not None else None,
                           used.data_ptr() if used is not None else None, ws.data_ptr(), wsb,
                           ctypes.c_void_p(ext.cuda_stream)))
            # ws (and the weights) are returned with the outputs so they stay alive until the caller drops the result
            return dict(bits=bits, soft=sft, iters_used=used, workspace=ws, weights=_wkeep)
        if is_torch:
            llr = llr.detach().cpu().numpy()
        x = np.ascontiguousarray(llr, dtype=fdt)
        if x.ndim != 2 or x.shape[1] != self.n:
            raise RuntimeError(f"llr must be (B, {self.n}), got {x.shape}")
        B = x.shape[0]
        bits = np.empty((B, self.n), np.uint8) if want_bits else None
        sft = np.empty((B, self.n), fdt) if soft else None
        used = np.empty((B,), np.int32) if want_iters else None
        if wstruct is not None:  # the weights were uploaded on the current torch stream; the library uses 0
            _torch().cuda.synchronize(self.device)
        check(call(x.ctypes.data, B, bits.ctypes.data if bits is not None else None,
                   sft.ctypes.data if sft is not None else None,
                   used.ctypes.data if used is not None else None, None, 0, None))
        return dict(bits=bits, soft=sft, iters_used=used)


_cache: dict = {}
_cache_lock = threading.Lock()


def get_decoder(H, device: int = 0) -> Decoder:
    """Graphs are built once per (H, device) — the reference rebuilt its dense masks on every
    decode_bits call (ofdm_functions.py:143/145)."""
    if isinstance(H, SparseCode):
        key = (H.shape, hashlib.sha1(H.row_ptr.tobytes() + H.col_idx.tobytes()).hexdigest(), int(device))
    else:
        H = np.asarray(H)
        key = (H.shape, hashlib.sha1(np.packbits(H.astype(np.uint8) & 1).tobytes()).hexdigest(), int(device))
    with _cache_lock:
        d = _cache.get(key)
        if d is None:
            d = Decoder(H, device)
            _cache[key] = d
        return d


def decode(H, llr, max_iters: int, *, algo="tanh", clamp=10.0, alpha=1.0, beta=0.0, early_stop=False,
           precision="f32", out="bits", device=None, llr_sign="p1/p0", **kw):
    """``decode(H, llr, max_iters)`` -> hard bits (uint8, (B, n)); ``out="bits+soft"`` -> (bits, p1).

    ``llr_sign``: "p1/p0" (default) = log P(1)/P(0), the reference's convention (ofdm_functions.py:72);
    "p0/p1" = the usual communications convention (positive = bit 0), negated once before decoding (an
    extra elementwise pass; results are those of the negated input)."""
    if llr_sign not in ("p1/p0", "p0/p1"):
        raise ValueError("llr_sign must be 'p1/p0' or 'p0/p1'")
    if llr_sign == "p0/p1":
        llr = -llr
    on_gpu = type(llr).__module__.startswith("torch") and llr.is_cuda
    if device is None:
        device = llr.device.index if on_gpu else 0
    elif on_gpu and int(device) != llr.device.index:
        raise ValueError(f"device={device} but llr is on {llr.device}")
    dec = get_decoder(H, device or 0)
    soft = "p1" if out == "bits+soft" else kw.pop("soft", None)
    r = dec.decode(llr, max_iters, algo=algo, clamp=clamp, alpha=alpha, beta=beta, early_stop=early_stop,
                   precision=precision, soft=soft, **kw)
    if out == "bits+soft":
        return r["bits"], r["soft"]
    if out == "bits":
        return r["bits"]
    return r


class _OutputPool:
    """Recycled float64 output buffers for ``decode_bits``.

    The reference's contract returns a fresh (N, n) float64 array per call (``ofdm_functions.py:133``); the
    host cost of a fresh 340 MB array is populating its pages (14-26 ms on the GPU box, more than the whole
    decode — DESIGN.md §9).  A returned array is an ordinary numpy array over a pooled buffer; when the caller
    drops it (and every view of it), a ``weakref.finalize`` on its per-call buffer exporter puts the buffer
    back, and a later call of the same size reuses it: the library rewrites every decoded row and the tail
    rows are zeroed, so each result is indistinguishable from a fresh ``np.zeros`` one.  At most ``keep`` free
    buffers of at most ``max_bytes`` in total are held (the oldest are released first).

    The finalizer can run inside ANY allocation on this thread (the cyclic GC frees an array that sat in a
    reference cycle), including while ``array()`` holds the pool's lock, so it takes no lock: it only appends
    to a deque (atomic), and ``array()`` folds the returned buffers into the free list under the lock."""

    def __init__(self, keep=2, max_bytes=2 << 30):
        import collections
        self.keep, self.max_bytes = keep, max_bytes
        self._free = []          # [(nbytes, 1-D float64 buffer)], oldest first; guarded by _lock
        self._returned = collections.deque()   # buffers handed back by finalizers (lock-free append)
        self._lock = threading.Lock()

    def _release(self, buf):
        self._returned.append(buf)   # no lock, no allocation beyond the deque slot: safe inside a GC pass

    def _fold(self):
        """Move returned buffers into the free list, oldest first, trimming to the limits (lock held)."""
        while True:
            try:
                buf = self._returned.popleft()
            except IndexError:
                break
            self._free.append((buf.nbytes, buf))
        while len(self._free) > self.keep or sum(b for b, _ in self._free) > self.max_bytes:
            self._free.pop(0)

    def free_count(self):
        with self._lock:
            self._fold()
            return len(self._free)

    def array(self, shape, rows):
        """(shape) float64 array whose rows >= ``rows`` are zero; rows < ``rows`` are for the caller to fill."""
        import weakref
        count = int(np.prod(shape))
        buf = None
        with self._lock:
            self._fold()
            for i, (nb, b) in enumerate(self._free):
                if b.size == count:
                    buf = self._free.pop(i)[1]
                    break
        if buf is None:
            if count * 8 > self.max_bytes:
                return np.zeros(shape)
            buf = np.empty(count)
        # the returned array (and every view of it) bottoms out in a per-call ctypes exporter of the pooled
        # memory: numpy collapses view chains onto the exporter, so it dies only with the last view
        holder = (ctypes.c_double * count).from_address(buf.ctypes.data)
        weakref.finalize(holder, self._release, buf)
        out = np.frombuffer(holder, dtype=np.float64).reshape(shape)
        out[rows:] = 0.0
        return out


_outputs = _OutputPool()


def decode_bits(llrs, H, bp_iterations, batch_size, clamp_value, *, fresh_output=None):
    """Drop-in for ``decode_bits`` (``pytorch/ofdm/ofdm_functions.py:131-163``).

    Same arguments and conventions: ``llrs`` (N, n) in log P(1)/P(0), converted to float32 as the
    reference does (``:156``); tanh sum-product for ``bp_iterations`` flooding iterations with messages
    clamped to ``clamp_value``; returns float64 0.0/1.0 of shape (N, n) where only the first
    ``(N // batch_size) * batch_size`` rows are decoded and the remainder stays 0 (``:133-135``).

    Output ownership: by default the result is a numpy array over a RECYCLED buffer (``_OutputPool``):
    ``out.flags.owndata`` is False (its ``.base`` is a ctypes exporter), so ``out.resize()`` raises, and
    once the caller has dropped the array and every view of it, a later call may rewrite that memory — a
    raw pointer kept past that point (``out.ctypes.data``) is not owned.  Values, shape, dtype and
    writeability are those of the reference's fresh ``np.zeros`` result.  ``fresh_output=True`` (or the
    environment variable ``LDPC_FRESH_OUTPUT=1``) returns a freshly allocated, self-owning array instead,
    as the reference does, at the cost of populating new pages on every call.
    """
    llrs = np.asarray(llrs)
    num_batches = llrs.shape[0] // batch_size  # ZeroDivisionError for batch_size == 0, as the reference
    rows = num_batches * batch_size
    if rows == 0 or llrs.ndim != 2:
        output_bits = np.zeros(llrs.shape)
        if rows == 0:
            return output_bits
    elif fresh_output or (fresh_output is None and os.environ.get("LDPC_FRESH_OUTPUT", "") not in ("", "0")):
        output_bits = np.zeros(llrs.shape)
    else:
        output_bits = _outputs.array(llrs.shape, rows)  # rows >= `rows` zero; the library writes the rest
    hshape = H.shape if isinstance(H, SparseCode) else np.asarray(H).shape
    if llrs.ndim != 2 or llrs.shape[1] != hshape[1]:
        raise RuntimeError(f"llrs shape {llrs.shape} does not match H {hshape}")
    dec = get_decoder(H)
    x = np.ascontiguousarray(llrs, dtype=np.float64)
    p = dec.params(int(bp_iterations), "tanh", float(clamp_value))
    # float64 -> float32 staging, chunked H2D / decode / D2H on two streams and the 0/1 float64 expansion
    # all run inside the library (ldpc_decode_bits_host); rows past `rows` stay 0 as in the reference
    check(dec.lib.ldpc_decode_bits_host(dec._h, x.ctypes.data, rows, ctypes.byref(p), output_bits.ctypes.data,
                                        0, 0))
    return output_bits


decoder = decode_bits


def _make_bp_module():
    torch = _torch()
    nn = torch.nn

    class BeliefPropagation(nn.Module):
        """``bp/bp.py:19-62`` interface: ``BeliefPropagation(H, iterations)``, ``forward(x, llr, clamp)``
        returns ``p1 = 1 - sigmoid(z)`` (B, n); ``.double()`` switches to float64 arithmetic like the
        reference module; ``layer_size()`` = number of edges E.  ``x`` = initial c2v messages in check-order
        (every reference caller passes zeros, ``ofdm_functions.py:157``; non-zero x runs ldpc_decode_x0).

        Weighted ("neural") BP forward: ``set_weights(...)`` with the reference's dense per-layer
        ``input_weight`` / ``llr_weight`` tensors, or ``load_reference_state_dict(sd)`` with a reference
        module's ``state_dict()`` (keys ``layers.{i}.0.input_weight``, ``layers.{i}.0.llr_weight``,
        ``final_layer.0.input_weight``, ``final_layer.0.llr_weight``, ``bp_vc.py:99-107``).  They are kept
        in the compact layout (``Graph.compact_weights``); forward then runs the weighted kernels.
        Training (the autograd backward of ``bp_vc.py:34-58``) is out of scope."""

        def __init__(self, H, iterations):
            super().__init__()
            self.H = H if isinstance(H, SparseCode) else np.asarray(H)
            self.iterations = int(iterations)
            self.graph = Graph.from_H(self.H)
            self.layer_size_val = self.graph.E
            self.register_buffer("_dtype_probe", torch.zeros(1, dtype=torch.float32))
            self.weights = None

        def layer_size(self):
            return self.layer_size_val

        def set_weights(self, input_weights=None, llr_weights=None, final_input_weight=None, final_llr_weight=None):
            """Dense reference-layout weights (lists over iterations for the first two); None = ones."""
            def cvt(a):
                return None if a is None else (a.detach().cpu().double().numpy() if torch.is_tensor(a) else a)
            iw = None if input_weights is None else [cvt(a) for a in input_weights]
            lw = None if llr_weights is None else [cvt(a) for a in llr_weights]
            for seq in (iw, lw):
                if seq is not None and len(seq) != self.iterations:
                    raise ValueError(f"need {self.iterations} per-layer weights, got {len(seq)}")
            c = self.graph.compact_weights(iw, lw, cvt(final_input_weight), cvt(final_llr_weight))
            self.weights = {k: (None if v is None else torch.from_numpy(v)) for k, v in c.items()}
            return self

        def load_reference_state_dict(self, sd):
            """Weights from a reference ``BeliefPropagation.state_dict()`` (load it with
            ``torch.load(path, weights_only=True)``)."""
            it = range(self.iterations)
            iw = [sd.get(f"layers.{i}.0.input_weight") for i in it]
            lw = [sd.get(f"layers.{i}.0.llr_weight") for i in it]
            return self.set_weights(None if any(a is None for a in iw) else iw,
                                    None if any(a is None for a in lw) else lw,
                                    sd.get("final_layer.0.input_weight"), sd.get("final_layer.0.llr_weight"))

        def forward(self, x, llr, clamp_value):
            precision = "f64" if self._dtype_probe.dtype == torch.float64 else "f32"
            dev = llr.device.index if llr.is_cuda else (torch.cuda.current_device() if torch.cuda.is_available() else 0)
            d = get_decoder(self.H, dev or 0)
            x0 = x if (x is not None and bool(torch.count_nonzero(x))) else None
            if x0 is not None and not llr.is_cuda:
                # non-zero initial messages go through the device path: stage both to the GPU and back
                p1 = self.forward(x.to(f"cuda:{dev or 0}"), llr.to(f"cuda:{dev or 0}"), clamp_value)
                return p1.cpu()
            r = d.decode(llr, self.iterations, algo="tanh", clamp=float(clamp_value), precision=precision,
                         soft="p1", want_bits=False, weights=self.weights, x0=x0)
            p1 = r["soft"]
            if not llr.is_cuda:
                p1 = torch.from_numpy(p1)
            return p1

    return BeliefPropagation


_BP = None


def __getattr__(name):  # lazy so that importing ldpc_amd does not import torch
    global _BP
    if name == "BeliefPropagation":
        if _BP is None:
            _BP = _make_bp_module()
        return _BP
    raise AttributeError(name)
