"""click_amd -- MI355X (gfx950) HIP implementation of Click's Internet-checksum path.

The product is the C ABI in include/click_amd_cksum.h, implemented by the
hand-written kernels in click_amd/csrc and built into
click_amd/libclick_amd_cksum.so.  This package is the thin Python host side
over that ABI: torch provides device memory and streams (plumbing only).

    ctx = click_amd.Context(0)
    b = click_amd.Batch(arena, stride=1536, fixed_len=1500, n=N)
    status, sums = ctx.set_udp_checksum(b)

There is no CPU fallback: every call goes to the HIP library and raises
ClickAmdError when the library reports an error.
"""
from . import _abi
from ._abi import (CLK_OK, CLK_IP_MINISCULE_PACKET, CLK_IP_BAD_VERSION, CLK_IP_BAD_HLEN,  # noqa: F401
                   CLK_IP_BAD_IP_LEN, CLK_IP_BAD_CHECKSUM, CLK_IP_BAD_SADDR, CLK_L4_NOT_PROTO,
                   CLK_L4_BAD_LENGTH, CLK_L4_BAD_CHECKSUM, CLK_SET_OK, CLK_SET_OUTPUT1, CLK_SET_KILL)
import ctypes
import os

import numpy as np

__all__ = ["Context", "Batch", "ClickAmdError", "lib", "read_pcap", "Pcap"]


class ClickAmdError(RuntimeError):
    pass


def lib():
    return _abi.load()


def _ptr(t):
    return None if t is None else ctypes.c_void_p(t.data_ptr())


class Batch:
    """Struct-of-arrays packet batch resident on the device.

    base: uint8 device tensor (the byte arena); off: int64/uint64 device
    tensor of byte offsets or None (then packet i is at i*stride); length:
    int32/uint32 device tensor or None (then every packet has fixed_len
    bytes).  See clk_batch in include/click_amd_cksum.h."""

    def __init__(self, base, n, stride=0, fixed_len=0, off=None, length=None, max_len=0):
        self.base, self.off, self.length = base, off, length
        self.n, self.stride, self.fixed_len, self.max_len = int(n), int(stride), int(fixed_len), int(max_len)
        if n and off is None and stride and hasattr(base, "numel") and (n - 1) * stride + fixed_len > base.numel():
            raise ValueError("batch exceeds its arena")

    def c(self):
        b = _abi.clk_batch()
        # base: a device tensor, or an int device address (a registered host
        # region's device base, Context.host_register)
        b.base = (self.base if isinstance(self.base, int) else self.base.data_ptr()) if self.base is not None else None
        b.off = self.off.data_ptr() if self.off is not None else None
        b.stride = self.stride
        b.len = self.length.data_ptr() if self.length is not None else None
        b.fixed_len = self.fixed_len
        b.max_len = self.max_len
        b.n = self.n
        return b


class Pcap:
    """A tcpdump file read by clk_pcap_read (FromDump(FILENAME, FORCE_IP)):
    `arena` (page-aligned uint8 numpy array, so it can be registered for
    zero-copy), per record `off`, `caplen`, `wire_len`, `ts_ns` and `nh`
    (the IP header's offset in the record, -1 when FORCE_IP found none),
    and the file's `info` (clk_pcap_info as a dict)."""

    def __init__(self, arena, off, caplen, wire_len, ts_ns, nh, info):
        self.arena, self.off, self.caplen, self.wire_len, self.ts_ns, self.nh = arena, off, caplen, wire_len, ts_ns, nh
        self.info = info

    def ip_records(self):
        """Indices of the records FORCE_IP kept (FromDump's output 0)."""
        return np.nonzero(self.nh >= 0)[0]

    def ip_layout(self):
        """(off, length) of the kept records' IP packets within the arena:
        the SoA of a clk_batch over them (nh applied)."""
        k = self.ip_records()
        return (self.off[k] + self.nh[k].astype(np.uint64)).astype(np.uint64), \
            (self.caplen[k] - self.nh[k].astype(np.uint32)).astype(np.uint32)


def read_pcap(path, force_ip=True, max_records=None):
    """Read a tcpdump file through the library (include/click_amd_ingest.h)."""
    L = lib()
    info = _abi.clk_pcap_info()
    p = os.fsencode(path)
    rc = L.clk_pcap_read(p, 1 if force_ip else 0, None, 0, None, None, None, None, None, 0, ctypes.byref(info))
    if rc < 0:
        raise ClickAmdError(L.clk_last_error(None).decode())
    n = info.records if max_records is None else min(info.records, max_records)
    page = 4096
    raw = np.zeros(int(info.arena_bytes) + 2 * page, np.uint8)
    start = (-raw.ctypes.data) % page
    arena = raw[start:start + ((int(info.arena_bytes) + page - 1) // page) * page]
    off = np.zeros(max(n, 1), np.uint64)
    cap = np.zeros(max(n, 1), np.uint32)
    wl = np.zeros(max(n, 1), np.uint32)
    ts = np.zeros(max(n, 1), np.uint64)
    nh = np.zeros(max(n, 1), np.int32)
    rc = L.clk_pcap_read(p, 1 if force_ip else 0, arena.ctypes.data, arena.size, off.ctypes.data, cap.ctypes.data,
                         wl.ctypes.data, ts.ctypes.data, nh.ctypes.data, n, ctypes.byref(info))
    if rc < 0:
        raise ClickAmdError(L.clk_last_error(None).decode())
    d = {f: getattr(info, f) for f, _ in _abi.clk_pcap_info._fields_}
    d["stopped"] = L.clk_last_error(None).decode() if rc == 1 else None
    return Pcap(arena, off[:n], cap[:n], wl[:n], ts[:n], nh[:n], d)


class Context:
    """One clk_ctx (device + HIP stream).  Not re-entrant; one per thread.

    stream: "torch" (default) launches on torch's current stream of the
    device, so the kernels are ordered with the torch ops that fill and read
    the tensors; "own" uses the context's own non-blocking stream; or any
    torch stream / raw hipStream_t handle."""

    def __init__(self, device=0, stream="torch", lib_path=None):
        import torch
        self._torch = torch
        self.lib = lib() if lib_path is None else _abi.load(lib_path)
        self.device = device
        h = ctypes.c_void_p()
        self._check(self.lib.clk_ctx_create(device, ctypes.byref(h)), None)
        self.h = h
        if isinstance(stream, str) and stream == "torch":
            stream = torch.cuda.current_stream(device)
        if not (isinstance(stream, str) and stream == "own"):
            self.set_stream(stream)

    def _check(self, rc, h=True):
        if rc != 0:
            msg = self.lib.clk_last_error(self.h if h else None)
            raise ClickAmdError("click_amd error %d: %s" % (rc, (msg or b"").decode()))

    def close(self):
        if getattr(self, "h", None):
            self.lib.clk_ctx_destroy(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    # -- streams ---------------------------------------------------------------
    def set_stream(self, stream):
        """stream: a torch.cuda.Stream / ExternalStream, a raw handle, or None
        (HIP's null stream)."""
        raw = getattr(stream, "cuda_stream", stream)
        self._check(self.lib.clk_ctx_set_stream(self.h, ctypes.c_void_p(raw) if raw else None))

    def use_own_stream(self):
        self._check(self.lib.clk_ctx_set_stream(self.h, self.lib.clk_ctx_own_stream(self.h)))

    def stream_handle(self):
        return self.lib.clk_ctx_stream(self.h)

    def torch_stream(self):
        return self._torch.cuda.ExternalStream(self.stream_handle(), device="cuda:%d" % self.device)

    def sync(self):
        self._check(self.lib.clk_ctx_sync(self.h))

    def reserve(self, max_packets):
        self._check(self.lib.clk_ctx_reserve(self.h, int(max_packets)))

    def tune(self, **knobs):
        """Speed-only tuning (clk_ctx_tune): max_blocks, scatter_blocks,
        set_mode (-1 auto, 0 fused, 1 two-phase), stream_min, group,
        set_chunks, read_shape (clk_read_stream, bench), frag_flat_min
        (clk_ip_fragment's flat payload pass from this batch size).  No
        setting changes a result."""
        for k, v in knobs.items():
            self._check(self.lib.clk_ctx_tune(self.h, _abi.TUNE[k], int(v)))
        return self

    # -- helpers ---------------------------------------------------------------
    def _out(self, n, dtype):
        return self._torch.empty(max(n, 1), dtype=dtype, device="cuda:%d" % self.device)

    # -- checksum path (include/click_amd_cksum.h) -----------------------------
    def in_cksum(self, b, out=None):
        out = self._out(b.n, self._torch.uint16) if out is None else out
        cb = b.c()
        self._check(self.lib.clk_in_cksum(self.h, ctypes.byref(cb), _ptr(out)))
        return out[:b.n]

    def check_ip_header(self, b, offset=0, checksum=True, badsrc=None, gooddst=None, out=None):
        out = self._out(b.n, self._torch.uint8) if out is None else out
        cfg = _abi.clk_ip_check_cfg()
        cfg.offset, cfg.checksum = offset, 1 if checksum else 0
        cfg.badsrc, cfg.nbadsrc = (badsrc.data_ptr(), badsrc.numel()) if badsrc is not None else (None, 0)
        cfg.gooddst, cfg.ngooddst = (gooddst.data_ptr(), gooddst.numel()) if gooddst is not None else (None, 0)
        cb = b.c()
        self._check(self.lib.clk_check_ip_header(self.h, ctypes.byref(cb), ctypes.byref(cfg), _ptr(out)))
        return out[:b.n]

    def set_ip_checksum(self, b, status=None, sums=None, want_sums=True):
        status = self._out(b.n, self._torch.uint8) if status is None else status
        if sums is None and want_sums:
            sums = self._out(b.n, self._torch.uint16)
        cb = b.c()
        self._check(self.lib.clk_set_ip_checksum(self.h, ctypes.byref(cb), _ptr(status), _ptr(sums)))
        return status[:b.n], (sums[:b.n] if sums is not None else None)

    def check_udp_header(self, b, out=None):
        out = self._out(b.n, self._torch.uint8) if out is None else out
        cb = b.c()
        self._check(self.lib.clk_check_udp_header(self.h, ctypes.byref(cb), _ptr(out)))
        return out[:b.n]

    def set_udp_checksum(self, b, status=None, sums=None, want_sums=True):
        status = self._out(b.n, self._torch.uint8) if status is None else status
        if sums is None and want_sums:
            sums = self._out(b.n, self._torch.uint16)
        cb = b.c()
        self._check(self.lib.clk_set_udp_checksum(self.h, ctypes.byref(cb), _ptr(status), _ptr(sums)))
        return status[:b.n], (sums[:b.n] if sums is not None else None)

    def check_tcp_header(self, b, out=None):
        out = self._out(b.n, self._torch.uint8) if out is None else out
        cb = b.c()
        self._check(self.lib.clk_check_tcp_header(self.h, ctypes.byref(cb), _ptr(out)))
        return out[:b.n]

    def set_tcp_checksum(self, b, fixoff=False, status=None, sums=None, want_sums=True):
        status = self._out(b.n, self._torch.uint8) if status is None else status
        if sums is None and want_sums:
            sums = self._out(b.n, self._torch.uint16)
        cb = b.c()
        self._check(self.lib.clk_set_tcp_checksum(self.h, ctypes.byref(cb), 1 if fixoff else 0,
                                                  _ptr(status), _ptr(sums)))
        return status[:b.n], (sums[:b.n] if sums is not None else None)

    def check_icmp_header(self, b, out=None):
        out = self._out(b.n, self._torch.uint8) if out is None else out
        cb = b.c()
        self._check(self.lib.clk_check_icmp_header(self.h, ctypes.byref(cb), _ptr(out)))
        return out[:b.n]

    def dec_ip_ttl(self, b, multicast=True, status=None, sums=None, want_sums=True):
        status = self._out(b.n, self._torch.uint8) if status is None else status
        if sums is None and want_sums:
            sums = self._out(b.n, self._torch.uint16)
        cb = b.c()
        self._check(self.lib.clk_dec_ip_ttl(self.h, ctypes.byref(cb), 1 if multicast else 0,
                                            _ptr(status), _ptr(sums)))
        return status[:b.n], (sums[:b.n] if sums is not None else None)

    # -- IP output path ----------------------------------------------------------
    def update_in_cksum(self, b, sum_off, hw_off, new_hw, zero_fix=False, zero_lo=0, status=None, sums=None,
                        want_sums=True):
        """click_update_in_cksum (+ click_update_zero_in_cksum) in place:
        new_hw is a uint16 device tensor of the words stored at hw_off."""
        status = self._out(b.n, self._torch.uint8) if status is None else status
        if sums is None and want_sums:
            sums = self._out(b.n, self._torch.uint16)
        cfg = _abi.clk_cksum_update_cfg(sum_off, hw_off, 1 if zero_fix else 0, zero_lo)
        cb = b.c()
        self._check(self.lib.clk_update_in_cksum(self.h, ctypes.byref(cb), ctypes.byref(cfg), _ptr(new_hw),
                                                 _ptr(status), _ptr(sums)))
        return status[:b.n], (sums[:b.n] if sums is not None else None)

    def update_zero_in_cksum(self, b, sum_off, zero_lo=0, status=None, sums=None, want_sums=True):
        status = self._out(b.n, self._torch.uint8) if status is None else status
        if sums is None and want_sums:
            sums = self._out(b.n, self._torch.uint16)
        cb = b.c()
        self._check(self.lib.clk_update_zero_in_cksum(self.h, ctypes.byref(cb), sum_off, zero_lo, _ptr(status),
                                                      _ptr(sums)))
        return status[:b.n], (sums[:b.n] if sums is not None else None)

    def _out_cfg(self, my_ip=0, ts=0, my_addrs=None, mtu=0xFFFFFFFF):
        cfg = _abi.clk_ip_out_cfg()
        cfg.my_ip, cfg.ts, cfg.mtu = my_ip & 0xFFFFFFFF, ts & 0xFFFFFFFF, mtu & 0xFFFFFFFF
        cfg.my_addrs, cfg.n_my_addrs = (my_addrs.data_ptr(), my_addrs.numel()) if my_addrs is not None else (None, 0)
        return cfg

    def ip_gw_options(self, b, my_ip, ts=0, my_addrs=None, status=None, problem=None, sums=None, want_sums=True):
        """IPGWOptions; my_ip / ts / my_addrs as raw (network-order) words."""
        status = self._out(b.n, self._torch.uint8) if status is None else status
        problem = self._out(b.n, self._torch.uint8) if problem is None else problem
        if sums is None and want_sums:
            sums = self._out(b.n, self._torch.uint16)
        cfg, cb = self._out_cfg(my_ip, ts, my_addrs), b.c()
        self._check(self.lib.clk_ip_gw_options(self.h, ctypes.byref(cb), ctypes.byref(cfg), _ptr(status),
                                               _ptr(problem), _ptr(sums)))
        return status[:b.n], problem[:b.n], (sums[:b.n] if sums is not None else None)

    def fix_ip_src(self, b, my_ip, anno=None, sums=None, want_sums=True):
        if sums is None and want_sums:
            sums = self._out(b.n, self._torch.uint16)
        cfg, cb = self._out_cfg(my_ip), b.c()
        self._check(self.lib.clk_fix_ip_src(self.h, ctypes.byref(cb), ctypes.byref(cfg), _ptr(anno), _ptr(sums)))
        return sums[:b.n] if sums is not None else None

    def ip_output_combo(self, b, my_ip, mtu, ts=0, flags=None, port=None, problem=None, sums=None,
                        want_sums=True, want_problem=True):
        port = self._out(b.n, self._torch.uint8) if port is None else port
        if problem is None and want_problem:
            problem = self._out(b.n, self._torch.uint8)
        if sums is None and want_sums:
            sums = self._out(b.n, self._torch.uint16)
        cfg, cb = self._out_cfg(my_ip, ts, None, mtu), b.c()
        self._check(self.lib.clk_ip_output_combo(self.h, ctypes.byref(cb), ctypes.byref(cfg), _ptr(flags),
                                                 _ptr(port), _ptr(problem), _ptr(sums)))
        return port[:b.n], (problem[:b.n] if problem is not None else None), \
            (sums[:b.n] if sums is not None else None)

    # -- IPFragmenter ------------------------------------------------------------
    def ip_fragment(self, b, mtu, honor_df=True, new_id=None, arena=None, max_frags=0, port=None,
                    first_len=None, frag_first=None):
        """IPFragmenter over the batch.  arena: uint8 device tensor for the
        appended fragments (None: size it with a first call -- the result's
        `totals` says what the batch needs).  Returns a dict of device
        tensors: port, first_len, frag_first, frag_off, frag_len, frag_src,
        totals (int64[2]: fragments, arena bytes)."""
        t = self._torch
        dev = "cuda:%d" % self.device
        port = self._out(b.n, t.uint8) if port is None else port
        first_len = self._out(b.n, t.int32) if first_len is None else first_len
        frag_first = self._out(b.n, t.int64) if frag_first is None else frag_first
        totals = t.zeros(2, dtype=t.int64, device=dev)
        fo = t.empty(max(max_frags, 1), dtype=t.int64, device=dev)
        fl = t.empty(max(max_frags, 1), dtype=t.int32, device=dev)
        fs = t.empty(max(max_frags, 1), dtype=t.int32, device=dev)
        cfg = _abi.clk_frag_cfg()
        cfg.mtu, cfg.honor_df = mtu, 1 if honor_df else 0
        cfg.new_id = new_id.data_ptr() if new_id is not None else None
        out = _abi.clk_frag_out()
        out.arena = arena.data_ptr() if arena is not None else None
        out.arena_bytes = arena.numel() if arena is not None else 0
        out.frag_off, out.frag_len, out.frag_src = fo.data_ptr(), fl.data_ptr(), fs.data_ptr()
        out.max_frags = max_frags
        cb = b.c()
        self._check(self.lib.clk_ip_fragment(self.h, ctypes.byref(cb), ctypes.byref(cfg), _ptr(port),
                                             _ptr(first_len), _ptr(frag_first), ctypes.byref(out), _ptr(totals)))
        return dict(port=port[:b.n], first_len=first_len[:b.n], frag_first=frag_first[:b.n], frag_off=fo,
                    frag_len=fl, frag_src=fs, totals=totals)

    # -- zero-copy host memory -----------------------------------------------------
    def host_register(self, arr):
        """Register a host numpy array for zero-copy kernel access; returns
        the device base address (int) of its first byte."""
        dev = ctypes.c_void_p()
        self._check(self.lib.clk_host_register(self.h, ctypes.c_void_p(arr.ctypes.data), arr.nbytes,
                                               ctypes.byref(dev)))
        return dev.value

    def host_unregister(self, arr):
        self._check(self.lib.clk_host_unregister(self.h, ctypes.c_void_p(arr.ctypes.data)))

    # -- utilities ---------------------------------------------------------------
    def count_codes(self, codes, ncounts=8, counts=None):
        if counts is None:
            counts = self._torch.zeros(ncounts, dtype=self._torch.int64, device="cuda:%d" % self.device)
        self._check(self.lib.clk_count_codes(self.h, _ptr(codes), codes.numel(), _ptr(counts), ncounts))
        return counts

    def gen_packets(self, b, proto=17, seed=0x5EED, first_idx=0):
        cb = b.c()
        self._check(self.lib.clk_gen_packets(self.h, ctypes.byref(cb), proto, seed, first_idx))

    def gen_corrupt(self, b, seed=0xBAD, rate_log2=10, first_idx=None, lo=None, hi=0):
        """Flip one bit in 1 of 2^rate_log2 packets (clk_gen_corrupt, or
        clk_gen_corrupt_span when first_idx / lo / hi are given: the pick
        hashed on the global index first_idx + i, the byte drawn from
        [lo, min(hi, len_i))).  Calling it twice restores the batch."""
        cb = b.c()
        if first_idx is None and lo is None and not hi:
            self._check(self.lib.clk_gen_corrupt(self.h, ctypes.byref(cb), seed, rate_log2))
        else:
            self._check(self.lib.clk_gen_corrupt_span(self.h, ctypes.byref(cb), seed, first_idx or 0, rate_log2,
                                                      0xFFFFFFFF if lo is None else lo, hi))

    def copy_stream(self, dst, src, shape=0, nbytes=None, out=None):
        """clk_copy_stream (bench: the copy ceiling; shape 4 the IMIX Set's
        read-all, write-one-block-in-six pattern, in place on src)."""
        if out is None:
            out = self._torch.zeros(1, dtype=self._torch.int64, device="cuda:%d" % self.device)
        nbytes = src.numel() * src.element_size() if nbytes is None else nbytes
        self._check(self.lib.clk_copy_stream(self.h, _ptr(dst) if dst is not None else None, _ptr(src), nbytes, shape,
                                             _ptr(out)))
        return out

    def read_stream(self, t, nbytes=None, out=None):
        if out is None:
            out = self._torch.zeros(1, dtype=self._torch.int64, device="cuda:%d" % self.device)
        nbytes = t.numel() * t.element_size() if nbytes is None else nbytes
        self._check(self.lib.clk_read_stream(self.h, _ptr(t), nbytes, _ptr(out)))
        return out
