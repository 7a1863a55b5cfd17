#!/bin/bash
# r03h: PCIe ceilings of the box (H2D over 1/2/4 streams, D2H, both at once, chunked H2D, the kernel's
# own zero-copy reads) for the host-path roofline.
set -o pipefail
export TMPDIR=/tmp
out=gpurun_out/r03h
mkdir -p $out
timeout -k 10 300 python -u profiles/pcie_probe.py 256 > $out/pcie.log 2>&1
