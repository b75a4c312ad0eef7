"""CPU tests of the drop-in boundary: the library builds, loads, exports every
symbol include/click_amd_cksum.h declares, and the Python ctypes mirror has
the C struct layouts.  No compute calls (no GPU here)."""
import ctypes
import os
import re
import subprocess
import tempfile

import pytest

from click_amd import _abi, build

ROOT = build.ROOT
HEADER = os.path.join(ROOT, "include", "click_amd_cksum.h")
HEADERS = [HEADER, os.path.join(ROOT, "include", "click_amd_elements.h"), os.path.join(ROOT, "include", "click_amd_ingest.h")]


def declared_functions():
    names = set()
    for h in HEADERS:
        text = open(h).read()
        text = re.sub(r"/\*.*?\*/", "", text, flags=re.S)
        names |= set(re.findall(r"\b(clk_[a-z0-9_]+)\s*\(", text))
    return sorted(names)


def test_library_builds_for_gfx950():
    lib = build.build_library()
    assert os.path.exists(lib)
    out = subprocess.run(["/opt/rocm/lib/llvm/bin/llvm-objdump", "--offloading", lib],
                         capture_output=True, text=True)
    blob = open(lib, "rb").read()
    assert b"gfx950" in blob, out.stdout[-400:]


def test_library_exports_every_declared_symbol():
    lib = _abi.load()
    names = declared_functions()
    assert len(names) >= 26
    for name in names:
        assert hasattr(lib, name), name
        assert name in _abi.SIGNATURES, "ctypes binding lacks " + name
    assert lib.clk_abi_version() == 6


def test_codes_agree_with_header_and_oracle():
    text = open(HEADER).read()
    for name in ("CLK_IP_MINISCULE_PACKET", "CLK_IP_BAD_VERSION", "CLK_IP_BAD_HLEN", "CLK_IP_BAD_IP_LEN",
                 "CLK_IP_BAD_CHECKSUM", "CLK_IP_BAD_SADDR", "CLK_L4_NOT_PROTO", "CLK_L4_BAD_LENGTH",
                 "CLK_L4_BAD_CHECKSUM", "CLK_SET_OUTPUT1", "CLK_SET_KILL"):
        m = re.search(r"\b%s\s*=\s*(\d+)" % name, text)
        assert m and int(m.group(1)) == getattr(_abi, name), name
        src = open(os.path.join(ROOT, "oracle", "cksum_oracle.c")).read()
        alias = name.replace("CLK_L4_NOT_PROTO", "CLK_L4_NOT_PROTO")
        m2 = re.search(r"#define %s (\d+)" % alias, src)
        assert m2 and int(m2.group(1)) == getattr(_abi, name), name


def test_struct_layouts_match_c():
    prog = r'''
#include <stdio.h>
#include <stddef.h>
#include "click_amd_cksum.h"
#include "click_amd_ingest.h"
int main(void) {
  printf("%zu %zu %zu %zu %zu %zu %zu\n", sizeof(clk_batch), offsetof(clk_batch, off),
         offsetof(clk_batch, stride), offsetof(clk_batch, len), offsetof(clk_batch, fixed_len),
         offsetof(clk_batch, max_len), offsetof(clk_batch, n));
  printf("%zu %zu %zu %zu %zu %zu\n", sizeof(clk_ip_check_cfg), offsetof(clk_ip_check_cfg, checksum),
         offsetof(clk_ip_check_cfg, badsrc), offsetof(clk_ip_check_cfg, nbadsrc),
         offsetof(clk_ip_check_cfg, ngooddst), offsetof(clk_ip_check_cfg, gooddst));
  printf("%zu %zu %zu %zu %zu\n", sizeof(clk_ip_out_cfg), offsetof(clk_ip_out_cfg, ts),
         offsetof(clk_ip_out_cfg, my_addrs), offsetof(clk_ip_out_cfg, n_my_addrs), offsetof(clk_ip_out_cfg, mtu));
  printf("%zu %zu %zu\n", sizeof(clk_frag_cfg), offsetof(clk_frag_cfg, honor_df), offsetof(clk_frag_cfg, new_id));
  printf("%zu %zu %zu %zu %zu %zu\n", sizeof(clk_frag_out), offsetof(clk_frag_out, arena_bytes),
         offsetof(clk_frag_out, frag_off), offsetof(clk_frag_out, frag_len), offsetof(clk_frag_out, frag_src),
         offsetof(clk_frag_out, max_frags));
  printf("%zu %zu %zu %zu\n", sizeof(clk_pcap_info), offsetof(clk_pcap_info, force_ip),
         offsetof(clk_pcap_info, records), offsetof(clk_pcap_info, ip_records));
  return 0; }
'''
    with tempfile.TemporaryDirectory() as d:
        c = os.path.join(d, "l.c")
        open(c, "w").write(prog)
        subprocess.run(["gcc", "-I", os.path.dirname(HEADER), "-o", os.path.join(d, "l"), c], check=True)
        out = subprocess.run([os.path.join(d, "l")], capture_output=True, text=True, check=True).stdout.split("\n")
    b = [int(x) for x in out[0].split()]
    cfg = [int(x) for x in out[1].split()]
    oc = [int(x) for x in out[2].split()]
    fc = [int(x) for x in out[3].split()]
    fo = [int(x) for x in out[4].split()]
    pc = [int(x) for x in out[5].split()]
    P = _abi.clk_pcap_info
    assert pc == [ctypes.sizeof(P), P.force_ip.offset, P.records.offset, P.ip_records.offset]
    O, F, FO = _abi.clk_ip_out_cfg, _abi.clk_frag_cfg, _abi.clk_frag_out
    assert oc == [ctypes.sizeof(O), O.ts.offset, O.my_addrs.offset, O.n_my_addrs.offset, O.mtu.offset]
    assert fc == [ctypes.sizeof(F), F.honor_df.offset, F.new_id.offset]
    assert fo == [ctypes.sizeof(FO), FO.arena_bytes.offset, FO.frag_off.offset, FO.frag_len.offset,
                  FO.frag_src.offset, FO.max_frags.offset]
    B = _abi.clk_batch
    assert b == [ctypes.sizeof(B), B.off.offset, B.stride.offset, B.len.offset, B.fixed_len.offset,
                 B.max_len.offset, B.n.offset]
    C = _abi.clk_ip_check_cfg
    assert cfg == [ctypes.sizeof(C), C.checksum.offset, C.badsrc.offset, C.nbadsrc.offset,
                   C.ngooddst.offset, C.gooddst.offset]


def test_header_is_plain_c():
    """The boundary header compiles as C99 with no C++ or torch types."""
    with tempfile.TemporaryDirectory() as d:
        c = os.path.join(d, "h.c")
        open(c, "w").write('#include "click_amd_cksum.h"\n#include "click_amd_elements.h"\n#include "click_amd_ingest.h"\n'
                           'int main(void){return 0;}\n')
        subprocess.run(["gcc", "-std=c99", "-Wall", "-Werror", "-pedantic", "-I", os.path.dirname(HEADER),
                        "-c", "-o", os.path.join(d, "h.o"), c], check=True)
    text = open(HEADER).read()
    assert "torch" not in re.sub(r"/\*.*?\*/", "", text, flags=re.S)


def test_missing_library_fails_loudly(tmp_path):
    with pytest.raises(OSError):
        _abi.load(str(tmp_path / "nope.so"))


def test_c_example_builds():
    """examples/pcap_check.c uses only the C headers (+ the HIP runtime for
    its device arrays) and links against the library with -Werror."""
    exes = build.build_examples()
    assert all(os.access(e, os.X_OK) for e in exes)


def test_click_adapters_use_only_the_public_abi():
    """The Click element sources (click_integration/elements/hip, not
    compilable here: they need Click's generated <click/config.h>) call only
    functions and constants the public headers declare, and every adapter
    class is exported under the reference name (hipdropin.cc) and a HIP
    name (hipparity.cc)."""
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    inc = os.path.join(root, "include")
    declared = set()
    for h in os.listdir(inc):
        declared |= set(re.findall(r"\b(clk_\w+)\s*\(", open(os.path.join(inc, h)).read()))
        declared |= set(re.findall(r"\b(CLK_\w+)\b", open(os.path.join(inc, h)).read()))
    hip = os.path.join(root, "click_integration", "elements", "hip")
    used = set()
    for f in os.listdir(hip):
        text = re.sub(r"//[^\n]*", "", re.sub(r"/\*.*?\*/", "", open(os.path.join(hip, f)).read(), flags=re.S))
        used |= set(re.findall(r"\b(clk_\w+)\s*\(", text)) | set(re.findall(r"\b(CLK_\w+)\b", text))
    assert used and used <= declared, sorted(used - declared)
    dropin = open(os.path.join(hip, "hipdropin.cc")).read()
    parity = open(os.path.join(hip, "hipparity.cc")).read()
    ref_names = ["CheckIPHeader", "CheckIPHeader2", "SetIPChecksum", "CheckUDPHeader", "SetUDPChecksum",
                 "CheckTCPHeader", "SetTCPChecksum", "CheckICMPHeader", "DecIPTTL", "IPInputCombo", "IPGWOptions",
                 "FixIPSrc", "IPOutputCombo", "IPFragmenter"]
    hh = "".join(open(os.path.join(hip, f)).read() for f in os.listdir(hip) if f.endswith(".hh"))
    for n in ref_names:
        assert "EXPORT_ELEMENT(HIP%s)" % n in dropin and "EXPORT_ELEMENT(HIP%sX)" % n in parity, n
        # click-buildtool reads class names from single-line class_name() methods
        assert re.search(r'class HIP%s\b.*?\n\s*const char \*class_name\(\) const\s*\{ return "%s"; \}' % (n, n), hh,
                         re.S), n


def test_click_adapters_keep_the_reference_processing():
    """Each adapter declares the reference class's processing (agnostic
    classes stay agnostic, so an unchanged graph that pulls through them
    passes Click's push/pull check, router.cc:692): PROCESSING_A_AH for
    CheckIPHeader (checkipheader.hh:114), CheckUDPHeader
    (checkudpheader.hh:61), CheckTCPHeader (checktcpheader.hh:61),
    CheckICMPHeader (checkicmpheader.hh:59), DecIPTTL (decipttl.hh:52),
    SetUDPChecksum (setudpchecksum.hh:32), IPGWOptions (ipgwoptions.hh:43);
    AGNOSTIC (element.cc:1127) for SetIPChecksum, SetTCPChecksum, FixIPSrc,
    IPInputCombo; PUSH for IPOutputCombo (ipoutputcombo.hh:52) and
    IPFragmenter (ipfragmenter.hh:65).  Every adapter with a pull side
    implements pull() (HIPBatchElement::pull, over hipcore's pull())."""
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    hip = os.path.join(root, "click_integration", "elements", "hip")
    hh = "".join(open(os.path.join(hip, f)).read() for f in sorted(os.listdir(hip)) if f.endswith(".hh"))
    base = re.search(r"class HIPBatchElement\b.*?processing\(\) const\s*\{ return (\w+); \}", hh, re.S).group(1)
    assert base == "PROCESSING_A_AH"
    assert re.search(r"Packet \*pull\(int port\);", hh)
    want = {"CheckIPHeader": "PROCESSING_A_AH", "CheckUDPHeader": "PROCESSING_A_AH",
            "CheckTCPHeader": "PROCESSING_A_AH", "CheckICMPHeader": "PROCESSING_A_AH", "DecIPTTL": "PROCESSING_A_AH",
            "SetUDPChecksum": "PROCESSING_A_AH", "IPGWOptions": "PROCESSING_A_AH", "SetIPChecksum": "AGNOSTIC",
            "SetTCPChecksum": "AGNOSTIC", "FixIPSrc": "AGNOSTIC", "IPInputCombo": "AGNOSTIC", "IPOutputCombo": "PUSH",
            "IPFragmenter": "PUSH"}
    for n, proc in want.items():
        body = re.search(r"class HIP%s\b[^{]*\{(.*?)\n\};" % n, hh, re.S).group(1)
        m = re.search(r"processing\(\) const\s*\{ return (\w+); \}", body)
        assert (m.group(1) if m else base) == proc, n
    cc = open(os.path.join(hip, "hipbatch.cc")).read()
    assert "_core.pull(*this, state())" in cc and "_core.push(*this, t, p)" in cc and "PerThread &t = state();" in cc


@pytest.mark.parametrize("cls,conf,msg", [
    ("CheckIPHeader", "INTERFACES 18.26.4.1/24 18.26.7.1/24, OFFSET 14", None),
    ("IPGWOptions", "18.26.4.24", None), ("SetUDPChecksum", "", None), ("IPFragmenter", "300, HONOR_DF true", None),
    ("CheckIPHeader", "FOO 3", "e0: FOO: unknown argument"), ("CheckIPHeader", "OFFSET x", "e0: OFFSET: invalid number"),
    ("SetUDPChecksum", "3", "e0: too many arguments"), ("IPFragmenter", "MTU x", "e0: MTU: invalid number"),
    ("CheckIPHeader", "BATCH 0", "e0: BATCH: expected positive integer"),
    ("NoSuchElement", "", "unknown element class NoSuchElement")])
def test_configuration_check_without_a_gpu(cls, conf, msg):
    """clk_element_check_config parses a class's keywords with no context and
    no device (the Click adapter's configure() calls it, so a bad keyword is
    a configure-time error on any host, in the reference's Args wording)."""
    lib = _abi.load()
    r = lib.clk_element_check_config(cls.encode(), conf.encode(), b"e0", 2)
    if msg is None:
        assert r == 0, lib.clk_last_error(None)
    else:
        assert r == _abi.CLK_EINVAL and lib.clk_last_error(None).decode() == msg
