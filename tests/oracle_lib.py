"""ctypes binding of the CPU oracle (oracle/cksum_oracle.c) -- test infrastructure.

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg use this.
"""
import ctypes
import os
import subprocess

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
ORACLE = os.path.join(ROOT, "oracle", "libcksum_oracle.so")

(OP_IN_CKSUM, OP_CHECK_IP, OP_SET_IP, OP_CHECK_UDP, OP_SET_UDP, OP_CHECK_TCP, OP_SET_TCP, OP_CHECK_ICMP,
 OP_DEC_TTL) = range(9)
OPS = {"in_cksum": OP_IN_CKSUM, "check_ip": OP_CHECK_IP, "set_ip": OP_SET_IP, "check_udp": OP_CHECK_UDP,
       "set_udp": OP_SET_UDP, "check_tcp": OP_CHECK_TCP, "set_tcp": OP_SET_TCP, "check_icmp": OP_CHECK_ICMP,
       "dec_ttl": OP_DEC_TTL}

_P = ctypes.c_void_p
_lib = None


def load_oracle():
    global _lib
    if _lib is not None:
        return _lib
    src = os.path.join(ROOT, "oracle", "cksum_oracle.c")
    if not os.path.exists(ORACLE) or os.path.getmtime(ORACLE) < os.path.getmtime(src):
        subprocess.run(["make", "-s", "-C", os.path.join(ROOT, "oracle")], check=True)
    L = ctypes.CDLL(ORACLE)
    L.oracle_in_cksum.restype = ctypes.c_uint16
    L.oracle_in_cksum.argtypes = [ctypes.c_char_p, ctypes.c_int]
    L.oracle_in_cksum_pseudohdr_raw.restype = ctypes.c_uint16
    L.oracle_in_cksum_pseudohdr_raw.argtypes = [ctypes.c_uint32] * 3 + [ctypes.c_int] * 2
    L.oracle_in_cksum_pseudohdr_hard.restype = ctypes.c_uint16
    L.oracle_in_cksum_pseudohdr_hard.argtypes = [ctypes.c_uint32, ctypes.c_char_p, ctypes.c_int]
    L.oracle_in_cksum_pseudohdr.restype = ctypes.c_uint16
    L.oracle_in_cksum_pseudohdr.argtypes = [ctypes.c_uint32, ctypes.c_char_p, ctypes.c_int]
    L.oracle_update_in_cksum.restype = ctypes.c_uint16
    L.oracle_update_in_cksum.argtypes = [ctypes.c_uint16] * 3
    L.oracle_update_zero_in_cksum.restype = ctypes.c_uint16
    L.oracle_update_zero_in_cksum.argtypes = [ctypes.c_uint16, ctypes.c_char_p, ctypes.c_int]
    L.oracle_check_ip_header.restype = ctypes.c_int
    L.oracle_check_ip_header.argtypes = [_P, ctypes.c_uint32, ctypes.c_uint32, ctypes.c_int, _P, ctypes.c_int,
                                         _P, ctypes.c_int]
    L.oracle_batch.restype = ctypes.c_int
    L.oracle_batch.argtypes = [ctypes.c_int, _P, _P, ctypes.c_uint64, _P, ctypes.c_uint32, ctypes.c_uint64,
                               ctypes.c_int, _P, _P]
    L.oracle_gen_batch.restype = None
    L.oracle_gen_batch.argtypes = [_P, _P, ctypes.c_uint64, _P, ctypes.c_uint32, ctypes.c_uint64, ctypes.c_int,
                                   ctypes.c_uint64, ctypes.c_uint64]
    L.oracle_bench.restype = ctypes.c_double
    L.oracle_bench.argtypes = [ctypes.c_int, _P, ctypes.c_uint64, ctypes.c_uint32, ctypes.c_uint64,
                               ctypes.c_int, ctypes.c_int]
    L.oracle_splitmix64.restype = ctypes.c_uint64
    L.oracle_splitmix64.argtypes = [ctypes.c_uint64]
    L.oracle_ip_out_batch.restype = ctypes.c_int
    L.oracle_ip_out_batch.argtypes = [ctypes.c_int, _P, _P, ctypes.c_uint64, _P, ctypes.c_uint32, ctypes.c_uint64,
                                      _P, ctypes.c_uint32, _P, ctypes.c_int, ctypes.c_uint32, ctypes.c_uint32,
                                      _P, _P, _P]
    L.oracle_ip_fragment_batch.restype = ctypes.c_int
    L.oracle_ip_fragment_batch.argtypes = [_P, _P, ctypes.c_uint64, _P, ctypes.c_uint32, ctypes.c_uint64,
                                           ctypes.c_uint32, ctypes.c_int, _P, _P, _P, _P, _P, _P, _P, _P, _P]
    L.oracle_check_l4_at.restype = ctypes.c_int
    L.oracle_check_l4_at.argtypes = [ctypes.c_int, _P, ctypes.c_uint32, ctypes.c_uint32]
    L.oracle_set_l4_at.restype = ctypes.c_int
    L.oracle_set_l4_at.argtypes = [ctypes.c_int, _P, ctypes.c_uint32, ctypes.c_uint32, ctypes.c_int, ctypes.c_int]
    _lib = L
    return L


def ip_fragment(arena, n, mtu, honor_df=False, stride=0, fixed_len=0, off=None, length=None, new_id=None):
    """IPFragmenter over a numpy arena (first fragments rewritten in place).
    Returns dict(port, first_len, frag_first, frags: list of bytes, frag_src,
    frag_off, frag_len, arena_bytes)."""
    L = load_oracle()
    off = None if off is None else np.ascontiguousarray(off, np.uint64)
    length = None if length is None else np.ascontiguousarray(length, np.uint32)
    nid = None if new_id is None else np.ascontiguousarray(new_id, np.uint16)
    port = np.zeros(max(n, 1), np.uint8)
    first = np.zeros(max(n, 1), np.uint32)
    ffirst = np.zeros(max(n, 1), np.uint64)
    totals = np.zeros(2, np.uint64)
    scratch = arena.copy()                     # sizing pass: the packets are rewritten in place
    L.oracle_ip_fragment_batch(_np_ptr(scratch), _np_ptr(off), stride, _np_ptr(length), fixed_len, n, mtu,
                               int(honor_df), _np_ptr(nid), _np_ptr(port), _np_ptr(first), _np_ptr(ffirst),
                               None, None, None, None, _np_ptr(totals))
    nf, nb = int(totals[0]), int(totals[1])
    out = np.zeros(max(nb, 1), np.uint8)
    foff = np.zeros(max(nf, 1), np.uint64)
    flen = np.zeros(max(nf, 1), np.uint32)
    fsrc = np.zeros(max(nf, 1), np.uint32)
    L.oracle_ip_fragment_batch(_np_ptr(arena), _np_ptr(off), stride, _np_ptr(length), fixed_len, n, mtu,
                               int(honor_df), _np_ptr(nid), _np_ptr(port), _np_ptr(first), _np_ptr(ffirst),
                               _np_ptr(out), _np_ptr(foff), _np_ptr(flen), _np_ptr(fsrc), _np_ptr(totals))
    frags = [out[int(foff[k]):int(foff[k]) + int(flen[k])].tobytes() for k in range(nf)]
    return dict(port=port[:n], first_len=first[:n], frag_first=ffirst[:n], frags=frags, frag_src=fsrc[:nf],
                frag_off=foff[:nf], frag_len=flen[:nf], arena=out[:nb], arena_bytes=nb)


IP_OUT_OPS = {"ip_gw_options": 0, "fix_ip_src": 1, "ip_output_combo": 2}


def ip_out_batch(op, arena, n, stride=0, fixed_len=0, off=None, length=None, flags=None, my_ip=0,
                 my_addrs=None, ts=0, mtu=0xFFFFFFFF):
    """IPGWOptions / FixIPSrc / IPOutputCombo over a numpy arena (modified in
    place).  Returns (codes or ports uint8[n], problem offsets uint8[n],
    ip_sum uint16[n])."""
    L = load_oracle()
    codes = np.zeros(max(n, 1), np.uint8)
    prob = np.zeros(max(n, 1), np.uint8)
    sums = np.zeros(max(n, 1), np.uint16)
    off = None if off is None else np.ascontiguousarray(off, np.uint64)
    length = None if length is None else np.ascontiguousarray(length, np.uint32)
    flags = None if flags is None else np.ascontiguousarray(flags, np.uint8)
    ma = None if my_addrs is None else np.ascontiguousarray(my_addrs, np.uint32)
    rc = L.oracle_ip_out_batch(IP_OUT_OPS[op], _np_ptr(arena), _np_ptr(off), stride, _np_ptr(length), fixed_len, n,
                               _np_ptr(flags), my_ip & 0xFFFFFFFF, _np_ptr(ma), 0 if ma is None else len(ma),
                               ts & 0xFFFFFFFF, mtu & 0xFFFFFFFF, _np_ptr(codes), _np_ptr(prob), _np_ptr(sums))
    assert rc == 0
    return codes[:n], prob[:n], sums[:n]


def _np_ptr(a):
    return None if a is None else a.ctypes.data_as(_P)


def batch(op, arena, n, stride=0, fixed_len=0, off=None, length=None, arg=1):
    """Run an element over a numpy byte arena (modified in place for sets).
    Returns (codes uint8[n], sums uint16[n])."""
    L = load_oracle()
    codes = np.zeros(max(n, 1), np.uint8)
    sums = np.zeros(max(n, 1), np.uint16)
    off = None if off is None else np.ascontiguousarray(off, np.uint64)
    length = None if length is None else np.ascontiguousarray(length, np.uint32)
    rc = L.oracle_batch(OPS[op] if isinstance(op, str) else op, _np_ptr(arena), _np_ptr(off), stride,
                        _np_ptr(length), fixed_len, n, arg, _np_ptr(codes), _np_ptr(sums))
    assert rc == 0
    return codes[:n], sums[:n]


def gen(arena, n, stride=0, fixed_len=0, off=None, length=None, proto=17, seed=0x5EED, first_idx=0):
    L = load_oracle()
    off = None if off is None else np.ascontiguousarray(off, np.uint64)
    length = None if length is None else np.ascontiguousarray(length, np.uint32)
    L.oracle_gen_batch(_np_ptr(arena), _np_ptr(off), stride, _np_ptr(length), fixed_len, n, proto, seed, first_idx)


# oracle_digest legs (oracle/cksum_oracle.h) and the bench element each stands for
DG_LEGS = ["check_l4", "set_l4", "check_ip", "set_ip", "dec_ttl", "out_combo"]
DG_ELEMENT_LEG = {"CheckUDPHeader": "check_l4", "CheckTCPHeader": "check_l4", "SetUDPChecksum": "set_l4",
                  "SetTCPChecksum": "set_l4", "CheckIPHeader": "check_ip", "SetIPChecksum": "set_ip",
                  "DecIPTTL": "dec_ttl", "IPOutputCombo": "out_combo"}


class DigestCfg(ctypes.Structure):
    _fields_ = [("proto", ctypes.c_int), ("imix", ctypes.c_int), ("fixed_len", ctypes.c_uint32),
                ("legs", ctypes.c_uint32), ("seed", ctypes.c_uint64), ("first_idx", ctypes.c_uint64),
                ("n", ctypes.c_uint64), ("corrupt_seed", ctypes.c_uint64), ("corrupt_log2", ctypes.c_uint32),
                ("ip_lo", ctypes.c_uint32), ("ip_hi", ctypes.c_uint32), ("ttl_runs", ctypes.c_int),
                ("my_ip", ctypes.c_uint32), ("mtu", ctypes.c_uint32)]


class DigestLeg(ctypes.Structure):
    _fields_ = [(f, ctypes.c_uint64) for f in ("ok", "packets", "sum16", "xor16", "wsum16", "wcode")]


def digest(elements, proto, first_idx, n, fixed_len=0, imix=False, seed=0x5EED, corrupt_seed=0xBAD,
           corrupt_log2=10, ip_span=(12, 20), ttl_runs=0, my_ip=0x18041A12, mtu=1500, threads=1):
    """The oracle's digest of bench.py's work on global packets
    [first_idx, first_idx + n) (oracle_digest): {element: {ok, packets,
    sum16, xor16, wsum16, wcode}}."""
    L = load_oracle()
    L.oracle_digest.restype = ctypes.c_int
    L.oracle_digest.argtypes = [ctypes.POINTER(DigestCfg), _P, ctypes.c_int, ctypes.POINTER(DigestLeg)]
    c = DigestCfg()
    c.proto, c.imix, c.fixed_len = proto, 1 if imix else 0, fixed_len
    c.legs = 0
    for e in elements:
        c.legs |= 1 << DG_LEGS.index(DG_ELEMENT_LEG[e])
    c.seed, c.first_idx, c.n = seed, first_idx, n
    c.corrupt_seed, c.corrupt_log2, c.ip_lo, c.ip_hi = corrupt_seed, corrupt_log2, ip_span[0], ip_span[1]
    c.ttl_runs, c.my_ip, c.mtu = ttl_runs, my_ip & 0xFFFFFFFF, mtu
    out = (DigestLeg * len(DG_LEGS))()
    rc = L.oracle_digest(ctypes.byref(c), None, max(1, threads), out)
    if rc != 0:
        raise RuntimeError("oracle_digest rc %d" % rc)
    return {e: {f: int(getattr(out[DG_LEGS.index(DG_ELEMENT_LEG[e])], f)) for f, _ in DigestLeg._fields_}
            for e in elements}
