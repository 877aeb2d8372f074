"""Register budget of the hot kernels: the HIP build writes the compiler's per-kernel resource
report (textblaster_amd/native.py build_hip, -Rpass-analysis=kernel-resource-usage); every kernel
named in csrc/hip/resource_budget.json must stay within its VGPR spill count and occupancy. A
one-field change to the shared document context once tripled k_stage_analyze_blk's spills
(229 -> 646) and cost config 5 11 % without failing any numerics test."""
import json
import os
import re

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_hot_kernels_within_register_budget():
    from textblaster_amd import native

    if not os.path.exists(native.RESOURCES_JSON):
        pytest.skip("no resource report: run __graft_entry__.build() first")
    if os.path.getmtime(native.RESOURCES_JSON) < os.path.getmtime(os.path.join(ROOT, "csrc/hip/kernels.hip")):
        pytest.skip("resource report older than kernels.hip: rebuild")
    rep = json.load(open(native.RESOURCES_JSON))
    budget = {k: v for k, v in json.load(open(os.path.join(ROOT, "csrc/hip/resource_budget.json"))).items()
              if not k.startswith("_")}
    bad = []
    for name, lim in budget.items():
        # Itanium mangling: <length><identifier>, so k_stage_analyze_blk does not match _blk_pre
        pat = re.compile(rf"{len(name)}{re.escape(name)}")
        hits = [v for k, v in rep.items() if pat.search(k)]
        assert hits, f"kernel {name} missing from the resource report"
        for v in hits:
            spill = v.get("VGPRs Spill", 0)
            occ = v.get("Occupancy [waves/SIMD]", 0)
            if spill > lim["max_vgpr_spill"] or occ < lim["min_occupancy"]:
                bad.append((name, spill, occ, lim))
    assert not bad, bad


def test_resource_remark_parser():
    from textblaster_amd.native import parse_resource_remarks

    text = ("k.hip:1:1: remark: Function Name: _Z3foov [-Rpass-analysis=kernel-resource-usage]\n"
            "k.hip:1:1: remark:     VGPRs: 80 [-Rpass-analysis=kernel-resource-usage]\n"
            "k.hip:1:1: remark:     ScratchSize [bytes/lane]: 576 [-Rpass-analysis=kernel-resource-usage]\n"
            "k.hip:1:1: remark:     Occupancy [waves/SIMD]: 6 [-Rpass-analysis=kernel-resource-usage]\n"
            "k.hip:1:1: remark:     VGPRs Spill: 229 [-Rpass-analysis=kernel-resource-usage]\n")
    assert parse_resource_remarks(text) == {"_Z3foov": {"VGPRs": 80, "ScratchSize [bytes/lane]": 576,
                                                        "Occupancy [waves/SIMD]": 6, "VGPRs Spill": 229}}
