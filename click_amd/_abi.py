"""ctypes binding of include/click_amd_cksum.h (the product C ABI).

This is the Python equivalent of the binding a host program adds for the
library; the Click-side C++ binding is in INTEGRATION.md.  No CPU fallback:
if the shared library is missing or cannot be loaded this module raises.
"""
import ctypes
import os

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(_HERE, "libclick_amd_cksum.so")

# return codes / verdicts (include/click_amd_cksum.h)
CLK_SUCCESS = 0
CLK_EINVAL = -1
CLK_EHIP = -2
CLK_ENODEV = -3

CLK_OK = 0
CLK_IP_MINISCULE_PACKET = 1
CLK_IP_BAD_VERSION = 2
CLK_IP_BAD_HLEN = 3
CLK_IP_BAD_IP_LEN = 4
CLK_IP_BAD_CHECKSUM = 5
CLK_IP_BAD_SADDR = 6
CLK_L4_NOT_PROTO = 1
CLK_L4_BAD_LENGTH = 2
CLK_L4_BAD_CHECKSUM = 3
CLK_SET_OK = 0
CLK_SET_OUTPUT1 = 1
CLK_SET_KILL = 2
CLK_TTL_OK = 0
CLK_TTL_EXPIRED = 1
CLK_TTL_UNCHANGED = 2
CLK_GWOPT_OK = 0
CLK_GWOPT_ERROR = 1
# clk_tune_knob
TUNE = {"max_blocks": 1, "scatter_blocks": 2, "set_mode": 3, "stream_min": 4, "group": 5, "set_chunks": 6,
        "read_shape": 7, "frag_flat_min": 8, "frag_chunks": 9}


class clk_batch(ctypes.Structure):
    _fields_ = [
        ("base", ctypes.c_void_p),
        ("off", ctypes.c_void_p),
        ("stride", ctypes.c_uint64),
        ("len", ctypes.c_void_p),
        ("fixed_len", ctypes.c_uint32),
        ("max_len", ctypes.c_uint32),
        ("n", ctypes.c_uint64),
    ]


class clk_ip_check_cfg(ctypes.Structure):
    _fields_ = [
        ("offset", ctypes.c_uint32),
        ("checksum", ctypes.c_int32),
        ("badsrc", ctypes.c_void_p),
        ("nbadsrc", ctypes.c_uint32),
        ("ngooddst", ctypes.c_uint32),
        ("gooddst", ctypes.c_void_p),
    ]


class clk_ip_out_cfg(ctypes.Structure):
    _fields_ = [
        ("my_ip", ctypes.c_uint32),
        ("ts", ctypes.c_uint32),
        ("my_addrs", ctypes.c_void_p),
        ("n_my_addrs", ctypes.c_uint32),
        ("mtu", ctypes.c_uint32),
    ]


class clk_frag_cfg(ctypes.Structure):
    _fields_ = [
        ("mtu", ctypes.c_uint32),
        ("honor_df", ctypes.c_int32),
        ("new_id", ctypes.c_void_p),
    ]


class clk_frag_out(ctypes.Structure):
    _fields_ = [
        ("arena", ctypes.c_void_p),
        ("arena_bytes", ctypes.c_uint64),
        ("frag_off", ctypes.c_void_p),
        ("frag_len", ctypes.c_void_p),
        ("frag_src", ctypes.c_void_p),
        ("max_frags", ctypes.c_uint64),
    ]


class clk_pcap_info(ctypes.Structure):
    _fields_ = [
        ("linktype", ctypes.c_int32),
        ("nanosecond", ctypes.c_int32),
        ("swapped", ctypes.c_int32),
        ("force_ip", ctypes.c_int32),
        ("records", ctypes.c_uint64),
        ("arena_bytes", ctypes.c_uint64),
        ("ip_records", ctypes.c_uint64),
    ]


_P = ctypes.c_void_p
_BP = ctypes.POINTER(clk_batch)
_OP = ctypes.POINTER(clk_ip_out_cfg)


class clk_cksum_update_cfg(ctypes.Structure):
    _fields_ = [("sum_off", ctypes.c_uint32), ("hw_off", ctypes.c_uint32), ("zero_fix", ctypes.c_int32),
                ("zero_lo", ctypes.c_uint32)]

# name -> (restype, argtypes); every symbol include/*.h declares
SIGNATURES = {
    "clk_abi_version": (ctypes.c_int, []),
    "clk_device_count": (ctypes.c_int, []),
    "clk_ctx_create": (ctypes.c_int, [ctypes.c_int, ctypes.POINTER(_P)]),
    "clk_ctx_destroy": (ctypes.c_int, [_P]),
    "clk_ctx_set_stream": (ctypes.c_int, [_P, _P]),
    "clk_ctx_stream": (_P, [_P]),
    "clk_ctx_own_stream": (_P, [_P]),
    "clk_ctx_sync": (ctypes.c_int, [_P]),
    "clk_ctx_device": (ctypes.c_int, [_P]),
    "clk_ctx_reserve": (ctypes.c_int, [_P, ctypes.c_uint64]),
    "clk_ctx_tune": (ctypes.c_int, [_P, ctypes.c_int, ctypes.c_int64]),
    "clk_last_error": (ctypes.c_char_p, [_P]),
    "clk_in_cksum": (ctypes.c_int, [_P, _BP, _P]),
    "clk_check_ip_header": (ctypes.c_int, [_P, _BP, ctypes.POINTER(clk_ip_check_cfg), _P]),
    "clk_set_ip_checksum": (ctypes.c_int, [_P, _BP, _P, _P]),
    "clk_check_udp_header": (ctypes.c_int, [_P, _BP, _P]),
    "clk_set_udp_checksum": (ctypes.c_int, [_P, _BP, _P, _P]),
    "clk_check_tcp_header": (ctypes.c_int, [_P, _BP, _P]),
    "clk_set_tcp_checksum": (ctypes.c_int, [_P, _BP, ctypes.c_int, _P, _P]),
    "clk_check_icmp_header": (ctypes.c_int, [_P, _BP, _P]),
    "clk_dec_ip_ttl": (ctypes.c_int, [_P, _BP, ctypes.c_int, _P, _P]),
    "clk_update_in_cksum": (ctypes.c_int, [_P, _BP, ctypes.POINTER(clk_cksum_update_cfg), _P, _P, _P]),
    "clk_update_zero_in_cksum": (ctypes.c_int, [_P, _BP, ctypes.c_uint32, ctypes.c_uint32, _P, _P]),
    "clk_ip_gw_options": (ctypes.c_int, [_P, _BP, _OP, _P, _P, _P]),
    "clk_fix_ip_src": (ctypes.c_int, [_P, _BP, _OP, _P, _P]),
    "clk_ip_output_combo": (ctypes.c_int, [_P, _BP, _OP, _P, _P, _P, _P]),
    "clk_ip_fragment": (ctypes.c_int, [_P, _BP, ctypes.POINTER(clk_frag_cfg), _P, _P, _P,
                                       ctypes.POINTER(clk_frag_out), _P]),
    "clk_host_register": (ctypes.c_int, [_P, _P, ctypes.c_size_t, ctypes.POINTER(_P)]),
    "clk_host_unregister": (ctypes.c_int, [_P, _P]),
    "clk_host_lookup": (ctypes.c_int, [_P, ctypes.c_size_t, ctypes.POINTER(_P), ctypes.POINTER(ctypes.c_size_t),
                                       ctypes.POINTER(_P)]),
    "clk_count_codes": (ctypes.c_int, [_P, _P, ctypes.c_uint64, _P, ctypes.c_uint32]),
    "clk_pcap_read": (ctypes.c_int, [ctypes.c_char_p, ctypes.c_int, _P, ctypes.c_uint64, _P, _P, _P, _P, _P,
                                     ctypes.c_uint64, ctypes.POINTER(clk_pcap_info)]),
    "clk_pcap_force_ip": (ctypes.c_int32, [_P, ctypes.c_uint32, ctypes.c_int32]),
    "clk_gen_packets": (ctypes.c_int, [_P, _BP, ctypes.c_int, ctypes.c_uint64, ctypes.c_uint64]),
    "clk_gen_corrupt": (ctypes.c_int, [_P, _BP, ctypes.c_uint64, ctypes.c_uint32]),
    "clk_gen_corrupt_span": (ctypes.c_int, [_P, _BP, ctypes.c_uint64, ctypes.c_uint64, ctypes.c_uint32,
                                            ctypes.c_uint32, ctypes.c_uint32]),
    "clk_read_stream": (ctypes.c_int, [_P, _P, ctypes.c_uint64, _P]),
    "clk_copy_stream": (ctypes.c_int, [_P, _P, _P, ctypes.c_uint64, ctypes.c_int, _P]),
    # include/click_amd_elements.h
    "clk_element_create": (ctypes.c_int, [_P, ctypes.c_char_p, ctypes.c_char_p, ctypes.c_char_p, ctypes.c_int,
                                          ctypes.POINTER(_P)]),
    "clk_element_destroy": (ctypes.c_int, [_P]),
    "clk_element_last_error": (ctypes.c_char_p, [_P]),
    "clk_element_push": (ctypes.c_int, [_P, _P, ctypes.c_uint32, ctypes.c_int32, ctypes.c_uint64]),
    "clk_element_push_burst": (ctypes.c_int, [_P, _P, _P, _P, ctypes.c_uint64, ctypes.c_uint32]),
    "clk_element_push_anno": (ctypes.c_int, [_P, _P, ctypes.c_uint32, ctypes.c_int32, ctypes.c_uint32,
                                             ctypes.c_uint64]),
    "clk_element_results_aux": (ctypes.c_uint64, [_P, _P, _P, _P, _P, ctypes.c_uint64]),
    "clk_element_take_packet": (ctypes.c_int64, [_P, ctypes.c_uint32, _P, ctypes.c_size_t]),
    "clk_element_flush": (ctypes.c_int, [_P]),
    "clk_element_flush_async": (ctypes.c_int, [_P]),
    "clk_element_results": (ctypes.c_uint64, [_P, _P, _P, _P, ctypes.c_uint64]),
    "clk_element_abandon": (ctypes.c_uint64, [_P]),
    "clk_element_share_messages": (ctypes.c_int, [_P, _P]),
    "clk_element_hold_packets": (ctypes.c_int, [_P, ctypes.c_int]),
    "clk_element_push_th": (ctypes.c_int, [_P, _P, ctypes.c_uint32, ctypes.c_int32, ctypes.c_int32, ctypes.c_uint32,
                                           ctypes.c_uint64]),
    "clk_element_check_config": (ctypes.c_int, [ctypes.c_char_p, ctypes.c_char_p, ctypes.c_char_p, ctypes.c_int]),
    "clk_element_read_handler": (ctypes.c_int, [_P, ctypes.c_char_p, ctypes.c_char_p, ctypes.c_size_t]),
    "clk_element_take_messages": (ctypes.c_int, [_P, ctypes.c_char_p, ctypes.c_size_t]),
    "clk_chain_create": (ctypes.c_int, [_P, ctypes.c_int, _P]),
    "clk_chain_destroy": (ctypes.c_int, [_P]),
    "clk_chain_last_error": (ctypes.c_char_p, [_P]),
    "clk_chain_flush_async": (ctypes.c_int, [_P]),
    "clk_chain_push_anno": (ctypes.c_int, [_P, _P, ctypes.c_uint32, ctypes.c_int32, ctypes.c_uint32, ctypes.c_uint64]),
    "clk_chain_push_burst": (ctypes.c_int, [_P, _P, _P, _P, ctypes.c_uint64, ctypes.c_uint32]),
    "clk_chain_flush": (ctypes.c_int, [_P]),
    "clk_chain_abandon": (ctypes.c_uint64, [_P]),
    "clk_chain_report_passes": (ctypes.c_int, [_P, ctypes.c_uint64]),
    "clk_chain_results": (ctypes.c_uint64, [_P, _P, _P, _P, _P, _P, ctypes.c_uint64]),
    "clk_chain_stats": (ctypes.c_int, [_P, _P, ctypes.c_int]),
}

_lib = None
_variants = {}


def load(path=LIB_PATH):
    """Load the HIP library (raises OSError if it is missing: no fallback)."""
    global _lib
    if _lib is not None and path == LIB_PATH:
        return _lib
    if path in _variants:
        return _variants[path]
    if not os.path.exists(path):
        raise OSError("click_amd: %s is missing; run `python -m click_amd.build` "
                      "(there is no CPU fallback)" % path)
    lib = ctypes.CDLL(path)
    for name, (res, args) in SIGNATURES.items():
        fn = getattr(lib, name)
        fn.restype = res
        fn.argtypes = args
    if path == LIB_PATH:
        _lib = lib
    else:
        _variants[path] = lib
    return lib
