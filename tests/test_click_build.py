"""CPU checks of the Click-facing adapter compiled into Click's userlevel
driver (tools/click_scratch_build.sh; skipped when the binaries were not
built): the drop-in build registers the GPU elements under the reference
class names and keeps the reference's configure-time errors (lib/args.cc:472,
476; include/click/args.hh:1061), a host without a gfx950 GPU fails at
initialize() with the adapter's message and exits cleanly, and the stock
build forwards config 1's 600000 packets (test/userlevel/iprouter-01.clicktest:
57,243) through click_integration/conf/c1-forward.click."""
import os

import pytest

from tests import click_run

pytestmark = pytest.mark.skipif(not (click_run.binary("cpu") and click_run.binary("dropin") and
                                     click_run.binary("parity")),
                                reason="Click binaries not built (tools/click_scratch_build.sh)")
NO_GPU = not os.path.exists("/dev/kfd")


@pytest.mark.parametrize("conf,msg", [("CheckIPHeader(FOO 3)", "FOO: unknown argument"),
                                      ("CheckIPHeader(OFFSET x)", "OFFSET: invalid number"),
                                      ("SetUDPChecksum(3)", "too many arguments"),
                                      ("IPFragmenter(MTU x)", "MTU: invalid number")])
def test_configure_errors_as_reference(conf, msg):
    """Same configure-time error text from the drop-in as from the stock
    element, and a clean exit (no crash in cleanup after a failed configure)."""
    expr = "InfiniteSource(LIMIT 1) -> %s -> Discard" % conf
    for mode in ("cpu", "dropin"):
        rc, _, err = click_run.run(mode, expr=expr)
        assert rc == 1, (mode, rc, err)
        assert "While configuring" in err and msg in err, (mode, err)


@pytest.mark.skipif(not NO_GPU, reason="a GPU is present")
@pytest.mark.parametrize("mode,cls", [("dropin", "CheckIPHeader"), ("dropin", "SetUDPChecksum"),
                                      ("dropin", "IPFragmenter"), ("parity", "HIPCheckIPHeader")])
def test_gpu_class_registered(mode, cls):
    """The class name resolves to the GPU adapter: configure passes (the
    glue's keywords accepted, BATCH among them) and initialize() reports that
    there is no gfx950 GPU -- the stock element would initialize."""
    conf = "BATCH 4" if cls != "IPFragmenter" else "300, BATCH 4"
    rc, _, err = click_run.run(mode, expr="InfiniteSource(LIMIT 1) -> %s(%s) -> Discard" % (cls, conf))
    assert rc == 1, err
    assert "While initializing" in err and "no gfx950 GPU" in err, err


def test_parity_build_has_both():
    """The parity build keeps the CPU classes beside the HIP-prefixed ones;
    the drop-in build has no HIP-prefixed names."""
    rc, _, err = click_run.run("parity", expr="InfiniteSource(LIMIT 1, STOP true) -> CheckIPHeader -> Discard")
    assert rc == 0, err
    rc, _, err = click_run.run("dropin", expr="InfiniteSource(LIMIT 1) -> HIPCheckIPHeader -> Discard")
    assert rc == 1 and "HIPCheckIPHeader" in err, err


def test_stock_click_config1_forward():
    """Config 1 on the reference's own elements: every one of 600000 frames
    forwarded (the count iprouter-01 expects), none dropped."""
    rc, h, err = click_run.run("cpu", "c1-forward.click", handlers=("out.count", "bad.count", "redirect.count"))
    assert rc == 0, err
    assert h["out.count"] == "600000" and h["bad.count"] == "0" and h["redirect.count"] == "0", h
