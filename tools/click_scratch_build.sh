#!/bin/bash
# click_scratch_build.sh -- build Click's userlevel driver with the GPU element
# group (click_integration/elements/hip) in a SCRATCH copy of the reference,
# to compile and run the Click-facing adapter (SURVEY.md §7 step 8, §8(c);
# BASELINE.md §2's config-1 plan).  Not an oracle: nothing built here is a
# checker of the kernels, nothing of the reference is committed, and the
# product library (click_amd/libclick_amd_cksum.so) is linked in, not built
# from it.
#
#   tools/click_scratch_build.sh cpu      the reference as it is (config 1's CPU baseline)
#   tools/click_scratch_build.sh dropin   GPU classes under the REFERENCE names
#                                         (--enable-skip-elements of the CPU ones)
#   tools/click_scratch_build.sh parity   CPU classes + HIP-prefixed GPU classes
#                                         (ComparePackets graphs)
#   tools/click_scratch_build.sh cpu-mt / dropin-mt  the same with
#                                         --enable-user-multithread (click -j N)
#   tools/click_scratch_build.sh dropin-pg  the drop-in compiled with -pg (gprof's
#                                         samples of Click and the adapter; the
#                                         glue library is not sampled), symbols kept
#
# Trees go to $CLICK_SCRATCH/<mode> (default /tmp/clickbuild); each build's
# `click` is stripped and copied to click_integration/bin/click-<mode>
# (git-ignored; it travels to the GPU box with the tree) and its log to
# $CLICK_SCRATCH/<mode>.log.  Configure line as SURVEY.md Appendix B.
set -euo pipefail
mode=${1:?usage: click_scratch_build.sh cpu|dropin|parity}
REPO=$(cd "$(dirname "$0")/.." && pwd)
REF=${CLICK_REF:-/root/reference}
SCRATCH=${CLICK_SCRATCH:-/tmp/clickbuild}
JOBS=${JOBS:-8}
DROPIN_SKIP=CheckIPHeader,CheckIPHeader2,SetIPChecksum,CheckUDPHeader,SetUDPChecksum,CheckTCPHeader,SetTCPChecksum,CheckICMPHeader,DecIPTTL,IPInputCombo,IPGWOptions,FixIPSrc,IPOutputCombo,IPFragmenter,HIPParity

pg=()
case "$mode" in
cpu) extra=() ;;
dropin) extra=(--enable-hip "--enable-skip-elements=$DROPIN_SKIP") ;;
dropin-pg) extra=(--enable-hip "--enable-skip-elements=$DROPIN_SKIP"); pg=(CXXFLAGS="-g -O2 -pg" CFLAGS="-g -O2 -pg") ;;
cpu-mt) extra=(--enable-user-multithread) ;;
dropin-mt) extra=(--enable-user-multithread --enable-hip "--enable-skip-elements=$DROPIN_SKIP") ;;
dropin-prof)
    # the drop-in with tools/core_profile/preload_sampler.c linked in: with
    # SAMPLES=file it samples the main thread's PC (its own CPU-time timer,
    # so HIP's threads do not take the signals, as they take gprof's)
    extra=(--enable-hip "--enable-skip-elements=$DROPIN_SKIP")
    gcc -O2 -c "$REPO/tools/core_profile/preload_sampler.c" -o "$SCRATCH/sampler.o"
    pg=(LIBS="$SCRATCH/sampler.o -ldl -lrt") ;;
parity) extra=(--enable-hip --enable-skip-elements=HIPCheckIPHeader) ;;
*) echo "unknown mode $mode" >&2; exit 2 ;;
esac

tree="$SCRATCH/$mode"
log="$SCRATCH/$mode.log"
mkdir -p "$SCRATCH"
rm -rf "$tree"
cp -r "$REF" "$tree"
if [ "${mode#cpu}" = "$mode" ]; then
    [ -f "$REPO/click_amd/libclick_amd_cksum.so" ] || python3 -m click_amd.build
    cp -r "$REPO/click_integration/elements/hip" "$tree/elements/hip"
fi
cd "$tree"
{
    echo "== configure ($mode)"
    ./configure --disable-linuxmodule --disable-bsdmodule --enable-userlevel --disable-dynamic-linking \
        "${extra[@]}" "${pg[@]}" CPPFLAGS="-I$REPO/include" \
        LDFLAGS="$([ "$mode" = dropin-pg ] && echo "-pg ")-L$REPO/click_amd -L/opt/rocm/lib -Wl,-rpath,/root/repo/click_amd -Wl,-rpath,/opt/rocm/lib"
    echo "== make"
    make -j"$JOBS"
} > "$log" 2>&1 || { tail -40 "$log"; exit 1; }
mkdir -p "$REPO/click_integration/bin"
if [ "$mode" = dropin-pg ] || [ "$mode" = dropin-prof ]; then
    strip --strip-debug -o "$REPO/click_integration/bin/click-$mode" userlevel/click
else
    strip -o "$REPO/click_integration/bin/click-$mode" userlevel/click
fi
echo "$REPO/click_integration/bin/click-$mode"
