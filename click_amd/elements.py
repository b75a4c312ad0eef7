"""Python handle on the batched GPU checksum elements (include/click_amd_elements.h).

The element logic is C++ (click_amd/host/elements.cc); this is the binding
a Python host (tests, bench) uses, as the Click adapter in INTEGRATION.md is
the binding Click's tree uses.

    ctx = click_amd.Context(0)
    e = Element(ctx, "CheckIPHeader", "OFFSET 14, DETAILS true", noutputs=2)
    e.push(frame_bytes_ndarray, nh_offset=14, token=7)
    e.flush()
    for token, port, length in e.results(): ...
    e.read_handler("drop_details")
"""
import ctypes

import numpy as np

from . import _abi, ClickAmdError

PORT_OUT0, PORT_OUT1, PORT_KILL = 0, 1, -1
ANNO_FIX_IP_SRC, ANNO_BCAST = 0x1, 0x2       # CLK_ANNO_* (include/click_amd_elements.h)
AUX_CLONE = 0x80000000


def anno_paint(color):
    return (color & 0xFF) << 8


class ResultBuffers:
    """Preallocated result arrays for Element.results(bufs=...): a caller
    that pops batch after batch reuses them instead of allocating (and
    page-faulting) four arrays per call."""

    def __init__(self, cap):
        self.tok = np.empty(cap, np.uint64)
        self.port = np.empty(cap, np.int32)
        self.len = np.empty(cap, np.uint32)
        self.aux = np.empty(cap, np.uint32)
        self.tok.fill(0), self.port.fill(0), self.len.fill(0), self.aux.fill(0)     # touch the pages once
        self.ptrs = [a.ctypes.data_as(ctypes.c_void_p) for a in (self.tok, self.port, self.len, self.aux)]


class Element:
    def __init__(self, ctx, class_name, config="", name=None, noutputs=1):
        """ctx: a click_amd.Context, or None: the element makes its own
        context on the GPU its DEVICE keyword names (default 0)."""
        self.ctx = ctx
        self.lib = ctx.lib if ctx is not None else _abi.load()
        ch = ctx.h if ctx is not None else None
        h = ctypes.c_void_p()
        rc = self.lib.clk_element_create(ch, class_name.encode(), config.encode(),
                                         name.encode() if name else None, noutputs, ctypes.byref(h))
        self.rc = rc
        if rc != 0:
            err = ClickAmdError("%s(%s): %s" % (class_name, config, (self.lib.clk_last_error(ch) or b"").decode()))
            err.rc = rc
            raise err
        self.h = h
        self._keep = []          # host buffers that must outlive flush()

    def last_error(self):
        return (self.lib.clk_element_last_error(self.h) or b"").decode()

    def abandon(self):
        """Route every staged / in-flight packet as killed (clk_element_abandon)."""
        k = int(self.lib.clk_element_abandon(self.h))
        self._keep = []
        return k

    def share_messages(self, other):
        """Count this element's once-only chatter with other's
        (clk_element_share_messages): one reference element's glue elements
        on several threads speak once."""
        if self.lib.clk_element_share_messages(self.h, other.h) != 0:
            raise ValueError("clk_element_share_messages failed")
        return self

    def hold_packets(self, on=True):
        """The caller keeps each pushed packet unchanged until its result is
        popped (clk_element_hold_packets): long spans may then be gathered
        at the flush instead of in the push."""
        if self.lib.clk_element_hold_packets(self.h, 1 if on else 0) != 0:
            raise ValueError("clk_element_hold_packets failed")
        return self

    def close(self):
        if getattr(self, "h", None):
            self.lib.clk_element_destroy(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def push(self, buf, length=None, nh_offset=-1, token=0, anno=0):
        """buf: a writable uint8 numpy array (or view) holding the packet;
        anno: CLK_ANNO_* bits (FixIPSrc, IPOutputCombo)."""
        length = buf.size if length is None else length
        self._keep.append(buf)
        rc = self.lib.clk_element_push_anno(self.h, buf.ctypes.data_as(ctypes.c_void_p), length, nh_offset, anno,
                                            token)
        if rc < 0:
            raise ClickAmdError("push failed: %d" % rc)
        return rc == 1

    def push_th(self, ptr, length, nh_offset, th_offset, token=0, anno=0):
        """clk_element_push_th: th_offset = the transport header annotation's
        offset from ptr (-2 none, -1 unknown).  Returns the raw status."""
        return self.lib.clk_element_push_th(self.h, ctypes.c_void_p(ptr), length, nh_offset, th_offset, anno, token)

    def push_ptr(self, ptr, length, nh_offset=-1, token=0):
        rc = self.lib.clk_element_push(self.h, ctypes.c_void_p(ptr), length, nh_offset, token)
        if rc < 0:
            raise ClickAmdError("push failed: %d" % rc)
        return rc == 1

    def push_burst(self, ptrs, lengths, nh_offsets=None, first_token=0):
        """ptrs: uint64 array of packet addresses; lengths: uint32 array;
        nh_offsets: int32 array or None.  Flushes whenever the batch fills."""
        ptrs = np.ascontiguousarray(ptrs, np.uint64)
        lengths = np.ascontiguousarray(lengths, np.uint32)
        nh = None if nh_offsets is None else np.ascontiguousarray(nh_offsets, np.int32)
        rc = self.lib.clk_element_push_burst(self.h, ptrs.ctypes.data_as(ctypes.c_void_p),
                                             lengths.ctypes.data_as(ctypes.c_void_p),
                                             None if nh is None else nh.ctypes.data_as(ctypes.c_void_p),
                                             first_token, len(ptrs))
        if rc != 0:
            raise ClickAmdError("push_burst failed: %d (%s)" % (rc, self.last_error()))

    def flush(self):
        rc = self.lib.clk_element_flush(self.h)
        if rc != 0:
            err = ClickAmdError("flush failed: %d (%s)" % (rc, self.last_error()))
            err.rc = rc
            raise err
        self._keep = []

    def flush_async(self):
        """Route the batch in flight, launch the staged one, do not wait
        (the host buffers pushed since the previous flush must stay valid
        until the next flush)."""
        rc = self.lib.clk_element_flush_async(self.h)
        if rc != 0:
            raise ClickAmdError("flush_async failed: %d (%s)" % (rc, self.last_error()))

    def results(self, cap=1 << 20, aux=False, bufs=None):
        """(tokens, ports, lengths[, aux]) of every flushed packet, in order
        (popped `cap` at a time: pass about the number expected).  bufs: a
        ResultBuffers to pop into (reused across calls; the arrays returned
        are then views of it, valid until its next use)."""
        if bufs is not None:
            n = self.lib.clk_element_results_aux(self.h, bufs.ptrs[0], bufs.ptrs[1], bufs.ptrs[2], bufs.ptrs[3],
                                                 len(bufs.tok))
            r = (bufs.tok[:n], bufs.port[:n], bufs.len[:n], bufs.aux[:n])
            return r if aux else r[:3]
        out = []
        while True:
            t = np.empty(cap, np.uint64)
            p = np.empty(cap, np.int32)
            ln = np.empty(cap, np.uint32)
            ax = np.empty(cap, np.uint32)
            n = self.lib.clk_element_results_aux(self.h, t.ctypes.data_as(ctypes.c_void_p),
                                                 p.ctypes.data_as(ctypes.c_void_p),
                                                 ln.ctypes.data_as(ctypes.c_void_p),
                                                 ax.ctypes.data_as(ctypes.c_void_p), cap)
            out.append((t[:n], p[:n], ln[:n], ax[:n]))
            if n < cap:
                break
        r = tuple(np.concatenate([o[k] for o in out]) for k in range(4))
        return r if aux else r[:3]

    def take_packet(self, key):
        """Bytes of a new packet the element made (IPFragmenter fragments)."""
        n = self.lib.clk_element_take_packet(self.h, key, None, 0)
        if n < 0:
            raise ClickAmdError("no packet %d" % key)
        buf = ctypes.create_string_buffer(max(int(n), 1))
        self.lib.clk_element_take_packet(self.h, key, buf, len(buf))     # copies and releases it
        return buf.raw[:n]

    def read_handler(self, name):
        buf = ctypes.create_string_buffer(1 << 16)
        n = self.lib.clk_element_read_handler(self.h, name.encode(), buf, len(buf))
        if n < 0:
            raise ClickAmdError("no handler %s" % name)
        return buf.value.decode()

    def messages(self):
        buf = ctypes.create_string_buffer(1 << 20)
        self.lib.clk_element_take_messages(self.h, buf, len(buf))
        return [m for m in buf.value.decode().split("\n") if m]


class Chain:
    """Consecutive elements on one device-resident batch (clk_chain_*):
    members[k+1] takes members[k]'s output 0.  Each packet is staged once,
    each member's kernel runs over what the members before it passed, and
    each packet is routed once; results name the member they leave.

        ch = Chain([Element(ctx, "CheckIPHeader", "OFFSET 14", noutputs=2),
                    Element(ctx, "DecIPTTL", "", noutputs=2)])
        ch.push_burst(ptrs, lengths, nh_offsets)
        ch.flush()
        tok, member, port, length, aux = ch.results()
    """

    def __init__(self, members):
        self.members = list(members)
        self.lib = self.members[0].lib
        arr = (ctypes.c_void_p * len(self.members))(*[m.h.value for m in self.members])
        h = ctypes.c_void_p()
        rc = self.lib.clk_chain_create(ctypes.cast(arr, ctypes.c_void_p), len(self.members), ctypes.byref(h))
        if rc != 0:
            err = ClickAmdError((self.lib.clk_last_error(None) or b"").decode())
            err.rc = rc
            raise err
        self.h = h

    def last_error(self):
        return (self.lib.clk_chain_last_error(self.h) or b"").decode()

    def push_anno(self, ptr, length, nh_offset=-1, anno=0, token=0):
        rc = self.lib.clk_chain_push_anno(self.h, ctypes.c_void_p(ptr), length, nh_offset, anno, token)
        if rc < 0:
            raise ClickAmdError("push failed: %d (%s)" % (rc, self.last_error()))
        return rc == 1

    def push_burst(self, ptrs, lengths, nh_offsets=None, first_token=0):
        ptrs = np.ascontiguousarray(ptrs, np.uint64)
        lengths = np.ascontiguousarray(lengths, np.uint32)
        nh = None if nh_offsets is None else np.ascontiguousarray(nh_offsets, np.int32)
        rc = self.lib.clk_chain_push_burst(self.h, ptrs.ctypes.data_as(ctypes.c_void_p),
                                           lengths.ctypes.data_as(ctypes.c_void_p),
                                           None if nh is None else nh.ctypes.data_as(ctypes.c_void_p),
                                           first_token, len(ptrs))
        if rc != 0:
            raise ClickAmdError("push_burst failed: %d (%s)" % (rc, self.last_error()))

    def flush(self):
        rc = self.lib.clk_chain_flush(self.h)
        if rc != 0:
            err = ClickAmdError("flush failed: %d (%s)" % (rc, self.last_error()))
            err.rc = rc
            raise err

    def flush_async(self):
        """Double-buffered flush (clk_chain_flush_async)."""
        rc = self.lib.clk_chain_flush_async(self.h)
        if rc != 0:
            err = ClickAmdError("flush_async failed: %d (%s)" % (rc, self.last_error()))
            err.rc = rc
            raise err

    def abandon(self):
        """Kill every packet still in the chain (clk_chain_abandon); returns the count."""
        return int(self.lib.clk_chain_abandon(self.h))

    def results(self, cap=1 << 20):
        """(tokens, members, ports, lengths, aux) of every routed result, in order."""
        out = []
        while True:
            a = [np.empty(cap, t) for t in (np.uint64, np.int32, np.int32, np.uint32, np.uint32)]
            n = self.lib.clk_chain_results(self.h, *[x.ctypes.data_as(ctypes.c_void_p) for x in a], cap)
            out.append([x[:n] for x in a])
            if n < cap:
                break
        return tuple(np.concatenate([o[k] for o in out]) for k in range(5))

    def close(self):
        if getattr(self, "h", None):
            self.lib.clk_chain_destroy(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass
