"""ctypes binding of libtmgpu.so (include/tmverify.h).

Loads the in-tree build (tendermint_amd/_build/libtmgpu.so).  Fails loudly
when it is missing — there is no CPU fallback on the product path.
"""
from __future__ import annotations

import ctypes
import os
import subprocess
import threading

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
# TMV_LIB_PATH: an A/B build of the same library (tools/build_ab.sh) for
# measurement runs; the default is the in-tree build
LIB_PATH = os.environ.get("TMV_LIB_PATH") or os.path.join(_HERE, "_build", "libtmgpu.so")
HEADER_PATH = os.path.join(os.path.dirname(_HERE), "include", "tmverify.h")
HEADER_PATHS = [HEADER_PATH, os.path.join(os.path.dirname(_HERE), "include", "tmhost.h")]

TMV_ALL_VALID = 1
TMV_NOT_ALL = 0
TMV_ERR_ARG = -1
TMV_ERR_NO_DEVICE = -2
TMV_ERR_NOMEM = -3
TMV_ERR_LAUNCH = -4
TMV_SR_ADDERR_PUBKEY = -1
TMV_SR_ADDERR_SIG = -2
TMV_KIND_ED25519 = 0
TMV_KIND_SR25519 = 1
TMV_FLAG_KEY_CACHE = 1
TMV_FLAG_BATCH_EQUATION = 2
TMV_FLAG_PER_ENTRY = 4
TMV_BATCHOPT_STATS = 1
TMV_BATCHOPT_SUBCHECK_ON = 2
TMV_BATCHOPT_SUBCHECK_OFF = 4
TMV_KIND_MIXED = 2
TMV_VOTE_WITH_BLOCK = 0x80000000

# tmv_vote (include/tmverify.h), 16 bytes
VOTE_DTYPE = np.dtype([("ts_seconds", "<i8"), ("ts_nanos", "<i4"), ("tmpl", "<u4")])

# Every symbol include/tmverify.h declares (checked by tests/test_boundary.py).
EXPORTS = [
    "tmv_open", "tmv_open_logical", "tmv_close", "tmv_num_devices", "tmv_last_error", "tmv_version",
    "tmv_ed25519_verify_batch", "tmv_ed25519_verify", "tmv_sr25519_verify_batch",
    "tmv_verify_mixed_batch", "tmv_ed25519_verify_batch_device", "tmv_verify_mixed_batch_device",
    "tmv_verify_batch_ex", "tmv_key_cache_stats", "tmv_set_batch_options", "tmv_batch_stats",
    "tmv_subgroup_stats", "tmv_validator_set_hashes",
    "tmv_verify_mixed_batch_ex", "tmv_verify_batch_device_ex", "tmv_verify_batches_device",
    "tmv_verify_votes", "tmv_vote_sign_bytes_device", "tmv_merkle_roots",
    "tmv_kernel_timing", "tmv_kernel_timing_read", "tmv_metrics_read", "tmv_metrics_reset",
    # include/tmhost.h
    "tmv_batch_new", "tmv_batch_add", "tmv_batch_len", "tmv_batch_verify", "tmv_batch_free",
    "tmv_vote_sign_bytes", "tmv_vote_template_encode", "tmv_verify_commit", "tmv_verify_commits",
    "tmv_header_hashes", "tmv_light_verify_many", "tmv_light_verify", "tmv_verify_vote_batch",
]


class BatchRef(ctypes.Structure):
    """tmv_batch_ref (include/tmverify.h): one device-resident batch."""
    _fields_ = [("pk", ctypes.c_void_p), ("sig", ctypes.c_void_p), ("msg", ctypes.c_void_p),
                ("msg_off", ctypes.c_void_p), ("n", ctypes.c_uint32), ("msg_bytes", ctypes.c_uint32),
                ("status", ctypes.c_void_p)]


class Metrics(ctypes.Structure):
    """tmv_metrics (include/tmverify.h)."""
    _fields_ = [("calls", ctypes.c_uint64), ("signatures", ctypes.c_uint64), ("max_batch", ctypes.c_uint64),
                ("batch_eq_signatures", ctypes.c_uint64), ("host_signatures", ctypes.c_uint64),
                ("host_seconds", ctypes.c_double), ("h2d_bytes", ctypes.c_uint64), ("d2h_bytes", ctypes.c_uint64),
                ("groups", ctypes.c_uint64), ("groups_failed", ctypes.c_uint64),
                ("located_groups", ctypes.c_uint64), ("fallback_signatures", ctypes.c_uint64),
                ("key_cache_hits", ctypes.c_uint64), ("key_cache_misses", ctypes.c_uint64)]


class VoteTemplate(ctypes.Structure):
    """tmv_vote_template (include/tmverify.h): the shared segments of a commit's votes."""
    _fields_ = [("head", ctypes.c_void_p), ("head_len", ctypes.c_uint32), ("block", ctypes.c_void_p),
                ("block_len", ctypes.c_uint32), ("chain", ctypes.c_void_p), ("chain_len", ctypes.c_uint32)]


def vote_templates(segments):
    """[(head, block, chain) bytes] -> (ctypes array of VoteTemplate, keep-alive buffers)."""
    keep = []
    arr = (VoteTemplate * max(1, len(segments)))()
    for t, segs in enumerate(segments):
        ptrs = []
        for b in segs:
            buf = ctypes.create_string_buffer(bytes(b), max(1, len(b)))
            keep.append(buf)
            ptrs.append((ctypes.cast(buf, ctypes.c_void_p), len(b)))
        arr[t] = VoteTemplate(ptrs[0][0], ptrs[0][1], ptrs[1][0], ptrs[1][1], ptrs[2][0], ptrs[2][1])
    return arr, keep


class NativeError(RuntimeError):
    pass


def build() -> str:
    """Compile libtmgpu.so for gfx950 in-tree (hipcc cross-compiles without a GPU)."""
    subprocess.run(["make", "-s", "-C", os.path.join(_HERE, "csrc")], check=True)
    return LIB_PATH


_lib = None
_lib_lock = threading.Lock()


def lib() -> ctypes.CDLL:
    """Load libtmgpu.so; raises NativeError if it has not been built."""
    global _lib
    with _lib_lock:
        if _lib is not None:
            return _lib
        if not os.path.exists(LIB_PATH):
            raise NativeError(f"{LIB_PATH} missing: run tendermint_amd._native.build() "
                              "(there is no CPU fallback)")
        L = ctypes.CDLL(LIB_PATH)
        u8p = ctypes.POINTER(ctypes.c_uint8)
        i8p = ctypes.POINTER(ctypes.c_int8)
        u32p = ctypes.POINTER(ctypes.c_uint32)
        vp = ctypes.c_void_p
        L.tmv_open.restype = vp
        L.tmv_open.argtypes = [ctypes.c_uint32]
        L.tmv_open_logical.restype = vp
        L.tmv_open_logical.argtypes = [ctypes.c_uint32, ctypes.c_int]
        L.tmv_close.argtypes = [vp]
        L.tmv_num_devices.argtypes = [vp]
        L.tmv_last_error.restype = ctypes.c_char_p
        L.tmv_version.restype = ctypes.c_char_p
        L.tmv_ed25519_verify_batch.argtypes = [vp, u8p, u8p, u8p, u32p, ctypes.c_uint32, u8p]
        L.tmv_ed25519_verify.argtypes = [vp, u8p, u8p, ctypes.c_size_t, u8p, ctypes.c_size_t]
        L.tmv_sr25519_verify_batch.argtypes = [vp, u8p, u8p, u8p, u32p, ctypes.c_uint32, i8p]
        L.tmv_verify_mixed_batch.argtypes = [vp, u8p, u8p, u8p, u8p, u32p, ctypes.c_uint32, i8p]
        L.tmv_verify_batch_ex.argtypes = [vp, ctypes.c_uint8, ctypes.c_uint32, u8p, u8p, u8p, u32p, ctypes.c_uint32,
                                          i8p]
        L.tmv_key_cache_stats.argtypes = [vp, ctypes.POINTER(ctypes.c_uint64), ctypes.POINTER(ctypes.c_uint64),
                                          ctypes.POINTER(ctypes.c_uint32), ctypes.POINTER(ctypes.c_uint32)]
        L.tmv_set_batch_options.argtypes = [vp, ctypes.c_uint32, ctypes.c_uint32, u8p, ctypes.c_uint32]
        L.tmv_batch_stats.argtypes = [vp, ctypes.POINTER(ctypes.c_uint64), ctypes.POINTER(ctypes.c_uint64)]
        L.tmv_kernel_timing.argtypes = [vp, ctypes.c_int]
        L.tmv_kernel_timing_read.argtypes = [vp, ctypes.c_char_p, ctypes.POINTER(ctypes.c_double),
                                             ctypes.POINTER(ctypes.c_uint64)]
        L.tmv_subgroup_stats.argtypes = [vp, ctypes.POINTER(ctypes.c_uint64), ctypes.POINTER(ctypes.c_uint64)]
        L.tmv_validator_set_hashes.argtypes = [vp, u8p, u8p, ctypes.POINTER(ctypes.c_int64), u32p,
                                               ctypes.c_uint32, u8p]
        L.tmv_verify_mixed_batch_ex.argtypes = [vp, ctypes.c_uint32, u8p, u8p, u8p, u8p, u32p, ctypes.c_uint32, i8p]
        L.tmv_verify_batch_device_ex.argtypes = [vp, ctypes.c_int, ctypes.c_uint8, ctypes.c_uint32, vp, vp, vp, vp,
                                                 vp, ctypes.c_uint32, vp, vp]
        L.tmv_verify_batches_device.argtypes = [vp, ctypes.c_int, ctypes.c_uint8, ctypes.c_uint32,
                                                ctypes.POINTER(BatchRef), ctypes.c_uint32, vp]
        L.tmv_verify_votes.argtypes = [vp, ctypes.c_uint8, ctypes.c_uint32, ctypes.POINTER(VoteTemplate),
                                       ctypes.c_uint32, vp, u8p, u8p, ctypes.c_uint32, i8p]
        L.tmv_vote_sign_bytes_device.restype = ctypes.c_int64
        L.tmv_vote_sign_bytes_device.argtypes = [vp, ctypes.POINTER(VoteTemplate), ctypes.c_uint32, vp,
                                                 ctypes.c_uint32, u8p, ctypes.c_size_t, u32p]
        L.tmv_ed25519_verify_batch_device.argtypes = [vp, ctypes.c_int, vp, vp, vp, vp, ctypes.c_uint32, vp, vp]
        L.tmv_verify_mixed_batch_device.argtypes = [vp, ctypes.c_int, vp, vp, vp, vp, vp, ctypes.c_uint32, vp, vp]
        L.tmv_metrics_read.argtypes = [vp, ctypes.POINTER(Metrics)]
        L.tmv_metrics_reset.argtypes = [vp]
        _lib = L
        return L


def last_error() -> str:
    return lib().tmv_last_error().decode(errors="replace")


def version() -> str:
    """tmv_version(): the library's version with its build id (source
    digest and git HEAD compiled in by csrc/Makefile)."""
    return lib().tmv_version().decode(errors="replace")


def build_info() -> dict:
    """The loaded library's build id against the sources of this tree:
    src_match says whether libtmgpu.so was compiled from them
    (csrc/src_digest.py computes the same digest the Makefile compiled in)."""
    import importlib.util
    v = version()
    fields = dict(kv.split("=", 1) for kv in v.split() if "=" in kv)
    spec = importlib.util.spec_from_file_location("tmv_src_digest", os.path.join(_HERE, "csrc", "src_digest.py"))
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    tree = mod.digest()
    return {"version": v, "src_digest_compiled": fields.get("src"), "src_digest_tree": tree,
            "src_match": fields.get("src") == tree, "git_head_compiled": fields.get("git"),
            "library": LIB_PATH}


def _p(a: np.ndarray, t=ctypes.c_uint8):
    return a.ctypes.data_as(ctypes.POINTER(t))


class Context:
    """A tmv_ctx on the devices in ``device_mask`` (0 = all visible)."""

    def __init__(self, device_mask: int = 0, logical: int = 1):
        """logical > 1: test aid (tmv_open_logical), every GPU opened as that
        many logical devices."""
        self._lib = lib()
        self._h = (self._lib.tmv_open(device_mask) if logical == 1
                   else self._lib.tmv_open_logical(device_mask, logical))
        if not self._h:
            raise NativeError("tmv_open failed: " + last_error())

    @property
    def handle(self):
        return self._h

    def close(self):
        if self._h:
            self._lib.tmv_close(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def num_devices(self) -> int:
        return self._lib.tmv_num_devices(self._h)

    @staticmethod
    def _check(rc: int, what: str) -> int:
        if rc < 0:
            raise NativeError(f"{what} failed ({rc}): {last_error()}")
        return rc

    def ed25519_verify_batch(self, pk: np.ndarray, sig: np.ndarray, msg: np.ndarray, off: np.ndarray):
        n = len(off) - 1
        out = np.zeros(max(n, 1), np.uint8)
        msg = msg if len(msg) else np.zeros(1, np.uint8)
        pk = pk if len(pk) else np.zeros(1, np.uint8)
        sig = sig if len(sig) else np.zeros(1, np.uint8)
        rc = self._check(self._lib.tmv_ed25519_verify_batch(self._h, _p(pk), _p(sig), _p(msg),
                                                            _p(off, ctypes.c_uint32), n, _p(out)),
                         "tmv_ed25519_verify_batch")
        return rc == TMV_ALL_VALID, out[:n]

    def ed25519_verify(self, pk: bytes, msg: bytes, sig: bytes) -> bool:
        a = np.frombuffer(pk, np.uint8).copy()
        m = np.frombuffer(msg + b"\0", np.uint8).copy()
        s = np.frombuffer(sig + b"\0", np.uint8).copy()
        rc = self._check(self._lib.tmv_ed25519_verify(self._h, _p(a), _p(m), len(msg), _p(s), len(sig)),
                         "tmv_ed25519_verify")
        return rc == 1

    def sr25519_verify_batch(self, pk, sig, msg, off):
        n = len(off) - 1
        out = np.zeros(max(n, 1), np.int8)
        msg = msg if len(msg) else np.zeros(1, np.uint8)
        pk = pk if len(pk) else np.zeros(1, np.uint8)
        sig = sig if len(sig) else np.zeros(1, np.uint8)
        rc = self._check(self._lib.tmv_sr25519_verify_batch(self._h, _p(pk), _p(sig), _p(msg),
                                                            _p(off, ctypes.c_uint32), n,
                                                            _p(out, ctypes.c_int8)),
                         "tmv_sr25519_verify_batch")
        return rc == TMV_ALL_VALID, out[:n]

    def verify_mixed_batch(self, kind, pk, sig, msg, off):
        n = len(off) - 1
        out = np.zeros(max(n, 1), np.int8)
        msg = msg if len(msg) else np.zeros(1, np.uint8)
        kind = kind if len(kind) else np.zeros(1, np.uint8)
        pk = pk if len(pk) else np.zeros(1, np.uint8)
        sig = sig if len(sig) else np.zeros(1, np.uint8)
        rc = self._check(self._lib.tmv_verify_mixed_batch(self._h, _p(kind), _p(pk), _p(sig), _p(msg),
                                                          _p(off, ctypes.c_uint32), n, _p(out, ctypes.c_int8)),
                         "tmv_verify_mixed_batch")
        return rc == TMV_ALL_VALID, out[:n]

    def verify_batch_ex(self, key_kind: int, flags: int, pk, sig, msg, off):
        n = len(off) - 1
        out = np.zeros(max(n, 1), np.int8)
        msg = msg if len(msg) else np.zeros(1, np.uint8)
        pk = pk if len(pk) else np.zeros(1, np.uint8)
        sig = sig if len(sig) else np.zeros(1, np.uint8)
        rc = self._check(self._lib.tmv_verify_batch_ex(self._h, key_kind, flags, _p(pk), _p(sig), _p(msg),
                                                       _p(off, ctypes.c_uint32), n, _p(out, ctypes.c_int8)),
                         "tmv_verify_batch_ex")
        return rc == TMV_ALL_VALID, out[:n]

    def verify_votes(self, key_kind: int, flags: int, templates, votes, pk, sig):
        """tmv_verify_votes: templates = [(head, block, chain)], votes = VOTE_DTYPE array."""
        votes = np.ascontiguousarray(votes, VOTE_DTYPE)
        n = len(votes)
        arr, keep = vote_templates(templates)
        out = np.zeros(max(n, 1), np.int8)
        pk = pk if len(pk) else np.zeros(1, np.uint8)
        sig = sig if len(sig) else np.zeros(1, np.uint8)
        rc = self._check(self._lib.tmv_verify_votes(self._h, key_kind, flags, arr, len(templates),
                                                    votes.ctypes.data if n else None, _p(pk), _p(sig), n,
                                                    _p(out, ctypes.c_int8)), "tmv_verify_votes")
        del keep
        return rc == TMV_ALL_VALID, out[:n]

    def vote_sign_bytes_device(self, templates, votes):
        """The messages k_vote_signbytes writes for (templates, votes): (msg bytes, offsets)."""
        votes = np.ascontiguousarray(votes, VOTE_DTYPE)
        n = len(votes)
        arr, keep = vote_templates(templates)
        off = np.zeros(n + 1, np.uint32)
        vp = votes.ctypes.data if n else None
        total = self._check(self._lib.tmv_vote_sign_bytes_device(self._h, arr, len(templates), vp, n, None, 0,
                                                                 _p(off, ctypes.c_uint32)), "tmv_vote_sign_bytes_device")
        msg = np.zeros(max(total, 1), np.uint8)
        self._check(self._lib.tmv_vote_sign_bytes_device(self._h, arr, len(templates), vp, n, _p(msg), len(msg),
                                                         _p(off, ctypes.c_uint32)), "tmv_vote_sign_bytes_device")
        del keep
        return msg[:total].tobytes(), off

    def verify_mixed_batch_ex(self, flags: int, kind, pk, sig, msg, off):
        n = len(off) - 1
        out = np.zeros(max(n, 1), np.int8)
        msg = msg if len(msg) else np.zeros(1, np.uint8)
        kind = kind if len(kind) else np.zeros(1, np.uint8)
        pk = pk if len(pk) else np.zeros(1, np.uint8)
        sig = sig if len(sig) else np.zeros(1, np.uint8)
        rc = self._check(self._lib.tmv_verify_mixed_batch_ex(self._h, flags, _p(kind), _p(pk), _p(sig), _p(msg),
                                                             _p(off, ctypes.c_uint32), n, _p(out, ctypes.c_int8)),
                         "tmv_verify_mixed_batch_ex")
        return rc == TMV_ALL_VALID, out[:n]

    def kernel_timing(self, enable: bool) -> None:
        """Bracket later launches of the timed kernels with HIP timing events
        on their streams (tmv_kernel_timing)."""
        self._check(self._lib.tmv_kernel_timing(self._h, 1 if enable else 0), "tmv_kernel_timing")

    def kernel_timing_read(self, kernel: str) -> tuple[float, int]:
        """(summed duration in ms, launches) of `kernel` since the last read
        (tmv_kernel_timing_read; waits for the recorded launches)."""
        ms, cnt = ctypes.c_double(0), ctypes.c_uint64(0)
        self._check(self._lib.tmv_kernel_timing_read(self._h, kernel.encode(), ctypes.byref(ms), ctypes.byref(cnt)),
                    "tmv_kernel_timing_read")
        return ms.value, cnt.value

    def set_batch_options(self, group_log2: int = 0, window_bits: int = 0, seed: bytes | None = None,
                          stats: bool = False, subcheck: bool | None = None) -> None:
        """Batch-equation options (tmv_set_batch_options): group size 2^group_log2,
        window bits, a fixed ChaCha20 key (tests only; None = fresh randomness
        per call), group-verdict counting and sub-group bisection (None =
        the default policy)."""
        sp = None
        if seed is not None:
            if len(seed) != 32:
                raise ValueError("seed must be 32 bytes")
            self._seed_buf = np.frombuffer(seed, np.uint8).copy()
            sp = _p(self._seed_buf)
        opt = (TMV_BATCHOPT_STATS if stats else 0) | \
            ({True: TMV_BATCHOPT_SUBCHECK_ON, False: TMV_BATCHOPT_SUBCHECK_OFF}.get(subcheck, 0))
        self._check(self._lib.tmv_set_batch_options(self._h, group_log2, window_bits, sp, opt),
                    "tmv_set_batch_options")

    def validator_set_hashes(self, pk: np.ndarray, kind: np.ndarray, power: np.ndarray,
                             set_off: np.ndarray) -> np.ndarray:
        """ValidatorSet.Hash of each set (tmv_validator_set_hashes): (n_sets, 32) uint8."""
        n_sets = len(set_off) - 1
        out = np.zeros((max(n_sets, 1), 32), np.uint8)
        pk = np.ascontiguousarray(pk, np.uint8) if len(pk) else np.zeros(32, np.uint8)
        kind = np.ascontiguousarray(kind, np.uint8) if len(kind) else np.zeros(1, np.uint8)
        power = np.ascontiguousarray(power, np.int64) if len(power) else np.zeros(1, np.int64)
        set_off = np.ascontiguousarray(set_off, np.uint32)
        self._check(self._lib.tmv_validator_set_hashes(self._h, _p(pk), _p(kind), _p(power, ctypes.c_int64),
                                                       _p(set_off, ctypes.c_uint32), n_sets, _p(out)),
                    "tmv_validator_set_hashes")
        return out[:n_sets]

    def batch_stats(self):
        g, f = ctypes.c_uint64(), ctypes.c_uint64()
        self._check(self._lib.tmv_batch_stats(self._h, ctypes.byref(g), ctypes.byref(f)), "tmv_batch_stats")
        sg, sf = ctypes.c_uint64(), ctypes.c_uint64()
        self._check(self._lib.tmv_subgroup_stats(self._h, ctypes.byref(sg), ctypes.byref(sf)), "tmv_subgroup_stats")
        return {"groups": g.value, "failed": f.value, "subgroups": sg.value, "sub_failed": sf.value}

    def verify_batch_device_ex(self, device: int, key_kind: int, flags: int, d_kind: int, d_pk: int, d_sig: int,
                               d_msg: int, d_off: int, n: int, d_status: int, stream: int = 0) -> None:
        self._check(self._lib.tmv_verify_batch_device_ex(self._h, device, key_kind, flags, d_kind or None, d_pk,
                                                         d_sig, d_msg, d_off, n, d_status, stream or None),
                    "tmv_verify_batch_device_ex")

    def verify_batches_device(self, device: int, key_kind: int, flags: int, refs, stream: int = 0) -> None:
        """refs: sequence of BatchRef (device pointers)."""
        arr = (BatchRef * len(refs))(*refs)
        self._check(self._lib.tmv_verify_batches_device(self._h, device, key_kind, flags, arr, len(refs),
                                                        stream or None), "tmv_verify_batches_device")

    def key_cache_stats(self):
        h, m = ctypes.c_uint64(), ctypes.c_uint64()
        u, c = ctypes.c_uint32(), ctypes.c_uint32()
        self._check(self._lib.tmv_key_cache_stats(self._h, ctypes.byref(h), ctypes.byref(m), ctypes.byref(u),
                                                  ctypes.byref(c)), "tmv_key_cache_stats")
        return {"hits": h.value, "misses": m.value, "used": u.value, "capacity": c.value}

    def metrics(self) -> dict:
        """tmv_metrics: cumulative counters (plus verifies_per_s_host, the
        end-to-end rate of the host-buffer calls)."""
        m = Metrics()
        self._check(self._lib.tmv_metrics_read(self._h, ctypes.byref(m)), "tmv_metrics_read")
        d = {k: getattr(m, k) for k, _ in Metrics._fields_}
        d["verifies_per_s_host"] = d["host_signatures"] / d["host_seconds"] if d["host_seconds"] else 0.0
        return d

    def metrics_reset(self) -> None:
        self._check(self._lib.tmv_metrics_reset(self._h), "tmv_metrics_reset")

    def ed25519_verify_batch_device(self, device: int, d_pk: int, d_sig: int, d_msg: int, d_off: int, n: int,
                                    d_valid: int, stream: int = 0) -> None:
        self._check(self._lib.tmv_ed25519_verify_batch_device(self._h, device, d_pk, d_sig, d_msg, d_off, n,
                                                              d_valid, stream or None),
                    "tmv_ed25519_verify_batch_device")

    def verify_mixed_batch_device(self, device: int, d_kind: int, d_pk: int, d_sig: int, d_msg: int, d_off: int,
                                  n: int, d_status: int, stream: int = 0) -> None:
        self._check(self._lib.tmv_verify_mixed_batch_device(self._h, device, d_kind, d_pk, d_sig, d_msg, d_off, n,
                                                            d_status, stream or None),
                    "tmv_verify_mixed_batch_device")


_default_ctx = None
_ctx_lock = threading.Lock()


def default_context() -> Context:
    """Process-wide context on all visible GPUs (like voi's global verifier)."""
    global _default_ctx
    with _ctx_lock:
        if _default_ctx is None:
            _default_ctx = Context(0)
        return _default_ctx
