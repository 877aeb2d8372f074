"""Device tuning: the GPU path's operating points in one place.

Every field has a measured default; an operator overrides them with ONE environment variable,

    TB_TUNE="slots=2,streams=serial,long_doc_bytes=8192"

(comma-separated ``key=value``; booleans as 0/1), or per engine with ``Engine(..., tuning=...)``.
``run --slots`` / ``--batch-bytes`` set the same fields from the CLI. Unknown keys are an error, so
a typo never silently measures the default. The A/B evidence behind each default is cited next to
its field; README.md "Tuning" lists them.

Compile-time budgets (waves per EU of each kernel, ``TB_*_WPE`` in csrc/hip/kernels.hip) are not
runtime knobs: tools/build_variant.sh builds an A/B library and ``TB_HIP_LIB`` loads it.
"""
from __future__ import annotations

import dataclasses
import os
from typing import Mapping, Optional, Tuple


@dataclasses.dataclass(frozen=True)
class DeviceTuning:
    # -- batches and streams --
    batch_bytes: int = 384 << 20   # text bytes per device batch (scratch 80-176 B/byte per slot)
    slots: int = 0                 # batches in flight; 0: 3 when HBM allows, else 2 (profiles/r2_slots/)
    streams: str = "6"             # "6": per slot compute + side, shared H2D/D2H (profiles/r2_streams/);
    #                                "serial": one stream, exclusive kernel times (tools/gpu.sh prof)
    blk_priority: int = -1         # HIP priority of the side (long-document) streams
    zero_copy: bool = True         # pinned inputs DMA'd in place, no host staging copy
    copy_threads: int = 8          # host threads of the staging copies / D2H unpacking
    prefetch_thread: bool = True   # process_many submits from a helper thread
    # -- LDS slices (bytes per document / workgroup) --
    lds_bytes: int = 0             # stage wave slice; 0: 160 KB / (4 x waves per SIMD) (profiles/r8_wpe/)
    lds_bytes_c4: int = 2560       # C4 pass A wave slice (per-line arrays only)
    lds_bytes_blk: int = 49152     # long-document workgroups: three per CU
    lds_bytes_dup: int = 0         # k_gr_dup_split slice; 0: = lds_bytes_blk
    lds_bytes_split: int = 5120    # k_gr_split_wave: 8 waves/SIMD (2.68 vs 2.80 ms at 6 KB, profiles/r8_wpe/)
    # -- document routing thresholds (bytes) --
    long_doc_bytes: int = 4096     # one workgroup instead of one wave (profiles/r2_c5/long_doc_threshold.txt)
    split_doc_bytes: int = 32768   # n-gram orders in k_gr_dup_split (config 5: 147.6 -> 152 K docs/s, profiles/r8_c5/)
    pre_doc_bytes: int = 262144    # multi-workgroup pre-pass (k_pre_*): ~1 MB docs 1,001 -> 1,136 docs/s (profiles/r5_pre/)
    ngram_big_bytes: int = 1200    # wave documents above: one wave per n-gram order (k_gr_split_wave)
    ngram_block: bool = True       # wave documents below: one workgroup per document (k_gr_ngrams)
    pre_wcanon: bool = True        # pre-pass documents hash/canonicalise words in k_pre_wcanon
    scratch_rate: Tuple[int, int] = (0, 0)  # scratch bytes per text byte (one pass, split); 0: devplan.h
    # -- device work placement (off = the host does it; A/B and debugging) --
    gate: bool = True              # step gating: later passes skip documents an earlier pass filtered
    lid_gate: bool = True          # a language-id pass gates the stage kernels after it
    device_resolve: bool = True    # K16: records resolved and outputs compacted on the device
    device_tokens: bool = True     # trailing TokenCounter steps counted on the device (k_bpe_count)
    dict_marks: bool = True        # dictionary-script docs: host ICU word marks, stay on the device
    c4_line_stats: bool = True     # C4 pass A reads the stage kernels' line export
    event_blocking: bool = True    # host waits on HIP events sleep instead of spinning
    # -- profiling --
    phase_prof: bool = False       # per-document phase cycle counters (tools/gpu.sh prof)

    def replace(self, **kw) -> "DeviceTuning":
        return dataclasses.replace(self, **{k: v for k, v in kw.items() if v is not None})


_FIELDS = {f.name: f for f in dataclasses.fields(DeviceTuning)}


def _value(name: str, raw: str):
    default = getattr(DeviceTuning, name) if not isinstance(getattr(DeviceTuning, name, None), property) else None
    raw = raw.strip()
    if isinstance(default, bool):
        if raw not in ("0", "1", "true", "false"):
            raise ValueError(f"TB_TUNE {name}: expected 0/1, got {raw!r}")
        return raw in ("1", "true")
    if isinstance(default, int):
        mult = 1
        for suf, m in (("k", 1 << 10), ("m", 1 << 20), ("g", 1 << 30)):
            if raw.lower().endswith(suf):
                raw, mult = raw[:-1], m
        return int(raw) * mult
    if isinstance(default, tuple):
        a, b = (int(v) for v in raw.replace("x", ":").split(":"))
        return (a, b)
    return raw


def parse(spec: str, base: Optional[DeviceTuning] = None) -> DeviceTuning:
    """``key=value,...`` -> DeviceTuning (on top of ``base``)."""
    kw = {}
    for item in (spec or "").split(","):
        if not item.strip():
            continue
        if "=" not in item:
            raise ValueError(f"TB_TUNE: {item!r} is not key=value")
        k, v = item.split("=", 1)
        k = k.strip()
        if k not in _FIELDS:
            raise ValueError(f"TB_TUNE: unknown key {k!r} (known: {', '.join(sorted(_FIELDS))})")
        kw[k] = _value(k, v)
    t = dataclasses.replace(base or DeviceTuning(), **kw)
    if t.streams not in ("6", "serial"):
        raise ValueError("TB_TUNE streams must be 6 or serial")
    if not 0 <= t.lds_bytes <= 131072 or not 0 <= t.lds_bytes_c4 <= 131072 or not 0 <= t.lds_bytes_blk <= 131072:
        # the workgroup kernels also hold static LDS: a 160 KB dynamic slice fails to launch
        raise ValueError("TB_TUNE lds_bytes* must be in [0, 131072]")
    if not 0 <= t.lds_bytes_split <= 65536:
        raise ValueError("TB_TUNE lds_bytes_split must be in [0, 65536]")
    return t


def from_env(env: Optional[Mapping[str, str]] = None) -> DeviceTuning:
    return parse((env if env is not None else os.environ).get("TB_TUNE", ""))
