"""The built gfx950 ISA keeps the arithmetic contract (CPU-side, no GPU needed).

* No fused multiply-add in any FedAvg kernel: the reference rounds the product and the sum
  separately (fedavg.py:25, `c1.add_(w * p1)`), and an FMA mismatches half the elements of
  the GNLeNet golden case (test_oracle_golden.test_fma_would_break_parity).  The teacher-logit
  mean kernels are exempt: IEEE-correct division expands to v_div_fmas/v_fma steps.
* Every dtype has its streaming, multi-tensor and scalar kernels.
"""
import re

import pytest

import isa

pytestmark = pytest.mark.skipif(not isa.available(), reason="ROCm llvm-objdump not present")

_FUSED = re.compile(r"^(v_fma\w*|v_fmac\w*|v_pk_fma\w*|v_mad_f32|v_mad_legacy\w*|v_mac_f32\w*|v_fma_mix\w*)\b")


@pytest.fixture(scope="module")
def funcs():
    from accdfl_amd import _lib

    return isa.disassemble(_lib.build())


def test_no_fused_multiply_add_in_fedavg_kernels(funcs):
    wsum = {n: body for n, body in funcs.items() if "wsum_" in n}
    assert len(wsum) > 20
    for name, body in wsum.items():
        fused = [ins for ins in body if _FUSED.match(ins)]
        assert not fused, "%s contains %s" % (name, fused[:3])


def test_every_dtype_has_its_kernels(funcs):
    names = " ".join(funcs)
    for dt in range(4):  # DLA_F32, DLA_BF16, DLA_F16, DLA_F64
        assert re.search(r"wsum_stream_kernelILi%dE" % dt, names), dt
        assert re.search(r"wsum_multi_kernelILi%dE" % dt, names), dt
        assert re.search(r"wsum_scalar_kernelILi%dE" % dt, names), dt


def test_wide_asm_stores_are_padded(funcs):
    """Every inline-asm 16-byte sc1 store is followed by s_nop: a store of more than 8 bytes
    reads its data VGPRs after issue, and hipcc pads nothing after an asm statement, so the
    next VALU could overwrite the data before the store has read it."""
    n = 0
    for name, body in funcs.items():
        for i, ins in enumerate(body):
            if ins.startswith("global_store_dwordx4") and "sc1" in ins:
                n += 1
                assert i + 1 < len(body) and body[i + 1].startswith("s_nop"), (name, ins, body[i + 1:i + 2])
    assert n > 0


def test_north_star_kernel_streams_dwordx4(funcs):
    """The f32 8-peer kernel (the bench's) loads 16 B per lane per peer with nt and stores sc1."""
    ns = [b for n, b in funcs.items() if re.search(r"wsum_stream_kernelILi0ELi8ELi64ELi1ELb1ELi2ELb0E", n)]
    assert ns
    body = ns[0]
    loads = [i for i in body if i.startswith("global_load_dwordx4")]
    stores = [i for i in body if i.startswith("global_store_dwordx4")]
    assert len(loads) >= 8 and all(" nt" in i for i in loads)
    assert stores and all("sc1" in i for i in stores)


def test_bigtile_kernel_streams_dwordx4(funcs):
    """The fp32 8-peer big-tile kernel (north-star default): 16-byte nt loads, sc1 stores, no spills,
    and at most 256 VGPRs + a few AGPRs (the two-buffer schedule, not every peer's data hoisted)."""
    bt = [b for n, b in funcs.items() if re.search(r"wsum_bigtile_kernelILi0ELi8ELi16E", n)]
    assert bt
    body = bt[0]
    loads = [i for i in body if i.startswith("global_load_dwordx4")]
    stores = [i for i in body if i.startswith("global_store_dwordx4")]
    assert len(loads) >= 16 * 8 and all(" nt" in i for i in loads)
    assert stores and all("sc1" in i for i in stores)
    assert not [i for i in body if i.startswith("scratch_")]
    agprs = [int(x) for ins in body for x in re.findall(r"\ba\[?(\d+)", ins)]
    assert max(agprs + [0]) < 64
