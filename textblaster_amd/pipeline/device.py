"""Device (MI355X) execution of the record-producing and content-rewriting steps for one batch.

Per batch: the packed UTF-8 text (uint8 bytes + int64 offsets, the Arrow LargeUtf8 layout) is
staged into HBM once; every device stage then reads it in place. C4 passes produce the next
content version directly in HBM (sizes -> device scan -> scatter), so later stages never go
back to the host. Records, per-document flags and the final content version are copied back
once at the end of the batch.
"""
from __future__ import annotations

import dataclasses
from typing import Dict, List, Optional, Tuple

import numpy as np

from .. import native
from ..errors import DeviceError
from .plan import ExecPlan

SCRATCH_ALIGN = 256


def _torch_dtypes():
    import torch

    return {np.dtype(np.uint8).str: torch.uint8, np.dtype(np.int32).str: torch.int32,
            np.dtype(np.int64).str: torch.int64, np.dtype(np.uint16).str: torch.int16}


_TORCH_DTYPES = _torch_dtypes() if __import__('importlib').util.find_spec('torch') else {}


@dataclasses.dataclass
class DeviceResult:
    stage_recs: List[np.ndarray]            # per stage: int64 [width_total * ndocs]
    c4_recs: Dict[int, np.ndarray]          # step index -> int64 [7 * ndocs]
    versions: Dict[int, Tuple[np.ndarray, np.ndarray]]  # v >= 1 -> (bytes, offsets)
    flags: np.ndarray                       # uint32 [ndocs]; nonzero -> recompute on the CPU path
    timings: Dict[str, float]


class DeviceRunner:
    def __init__(self, steps_native, plan: ExecPlan, device, langid=None):
        import torch

        self.torch = torch
        self.device = torch.device(device)
        self.plan = plan
        self.steps = steps_native
        h = native.host()
        from ..ops.kernels import Kernels

        self.k = Kernels(torch, self.device)
        plan_b, stage_bs = h.build_device_plan(steps_native, plan.stages)
        self.plan_t = self._to_dev(plan_b)
        self.stage_ts = [self._to_dev(b) for b in stage_bs]
        self.stage_layout = [h.stage_layout(b) for b in stage_bs]
        self.c4_ts = {i: self._to_dev(h.build_c4(steps_native[i])) for i in plan.c4_steps}
        self.has_lid = any(steps_native[i].kind == h.StepKind.LanguageDetection for st in plan.stages for i in st)
        if self.has_lid:
            if langid is None:
                raise DeviceError("LanguageDetectionFilter needs a language-id model")
            self.lid_emb = torch.from_numpy(langid.emb).to(self.device)
            wT = np.ascontiguousarray(langid.w.reshape(h.LID_DIM, h.LID_LANGS_PAD).T)  # [16][32]
            self.lid_wT = torch.from_numpy(wT).to(self.device)
            self.lid_b = torch.from_numpy(langid.b.astype(np.float32)).to(self.device)
        self._scratch = None
        self._pinned = None
        self._last_lid = None

    def _to_dev(self, b: bytes):
        t = self.torch.frombuffer(bytearray(b), dtype=self.torch.uint8)
        return t.to(self.device)

    def _scratch_for(self, nbytes: int):
        if self._scratch is None or self._scratch.numel() < nbytes:
            self._scratch = None
            self._scratch = self.torch.empty(int(nbytes * 1.25) + (1 << 20), dtype=self.torch.uint8,
                                             device=self.device)
        return self._scratch

    def _h2d(self, arr: np.ndarray):
        # staged through a pinned host buffer so the copy is a DMA (and numpy read-only views
        # of Arrow buffers are never handed to torch directly)
        arr = np.ascontiguousarray(arr)
        nb = arr.nbytes
        if self._pinned is None or self._pinned.numel() < nb:
            self._pinned = self.torch.empty(max(nb, 1 << 20) * 2, dtype=self.torch.uint8, pin_memory=True)
        host = self._pinned[:nb]
        host.numpy()[:] = arr.view(np.uint8).reshape(-1)
        dev = self.torch.empty(nb, dtype=self.torch.uint8, device=self.device)
        dev.copy_(host, non_blocking=False)
        return dev.view(_TORCH_DTYPES[arr.dtype.str]) if nb else dev

    def run(self, data: np.ndarray, off: np.ndarray) -> DeviceResult:
        import time

        torch = self.torch
        h = native.host()
        t0 = time.perf_counter()
        ndocs = len(off) - 1
        lens = np.diff(off)
        perm = np.argsort(-lens, kind="stable").astype(np.int32)
        per_doc = (h.scratch_bytes_for(0) - 64 * 160) + 160 * (lens + 64)
        per_doc = (per_doc + SCRATCH_ALIGN - 1) // SCRATCH_ALIGN * SCRATCH_ALIGN
        scratch_off = np.zeros(ndocs + 1, dtype=np.int64)
        np.cumsum(per_doc, out=scratch_off[1:])
        scratch = self._scratch_for(int(scratch_off[-1]))
        maxlen = int(lens.max()) if ndocs else 0
        pw, pw_n = self.k.pow_table(2 * maxlen + 64)
        d_bytes = self._h2d(data if len(data) else np.zeros(1, np.uint8))
        d_off = self._h2d(off)
        d_perm = self._h2d(perm)
        d_soff = self._h2d(scratch_off)
        flags = torch.zeros(ndocs, dtype=torch.int32, device=self.device)
        t1 = time.perf_counter()
        versions = {0: (d_bytes, d_off, len(data))}
        stage_recs_d = []
        c4_recs_d = {}
        for ver in range(self.plan.n_versions):
            vb, vo, vlen = versions[ver]
            for s, sv in enumerate(self.plan.stage_version):
                if sv != ver:
                    continue
                width_total, layout = self.stage_layout[s]
                rec = torch.zeros(width_total * ndocs, dtype=torch.int64, device=self.device)
                lid_vec = lid_cnt = None
                if any(kind == 4 for kind, _, _ in layout):
                    lid_vec = torch.zeros(ndocs * h.LID_DIM, dtype=torch.int16, device=self.device)
                    lid_cnt = torch.zeros(ndocs, dtype=torch.int32, device=self.device)
                self.k.stage_analyze(self.plan_t, self.stage_ts[s], vb, vo, d_perm, ndocs, scratch, d_soff, pw, pw_n,
                                     rec, flags, self.lid_emb if lid_vec is not None else None, lid_vec, lid_cnt)
                if lid_vec is not None:
                    self._last_lid = (lid_vec, lid_cnt)
                for kind, width, prefix in layout:
                    if kind == 4:
                        self.k.langid_head(lid_vec, lid_cnt, self.lid_wT, self.lid_b, ndocs, rec, prefix * ndocs, width)
                stage_recs_d.append((s, rec))
            c4_here = [i for i in self.plan.c4_steps if self.plan.steps[i].version_in == ver]
            for i in c4_here:
                rec = torch.zeros(7 * ndocs, dtype=torch.int64, device=self.device)
                src = torch.zeros(2 * ndocs, dtype=torch.int64, device=self.device)
                self.k.c4_pass_a(self.c4_ts[i], vb, vo, d_perm, ndocs, scratch, d_soff, pw, pw_n, rec, src, flags)
                new_off = torch.zeros(ndocs + 1, dtype=torch.int64, device=self.device)
                torch.cumsum(src.view(ndocs, 2)[:, 1], 0, out=new_off[1:])
                cap = 2 * vlen + ndocs + 16
                out = torch.empty(cap, dtype=torch.uint8, device=self.device)
                self.k.c4_pass_b(vb, vo, ndocs, scratch, d_soff, src, new_off, out)
                versions[ver + 1] = (out, new_off, cap)
                c4_recs_d[i] = rec
        torch.cuda.synchronize(self.device)
        t2 = time.perf_counter()
        stage_recs = [None] * len(self.plan.stages)
        for s, rec in stage_recs_d:
            stage_recs[s] = rec.cpu().numpy()
        c4_recs = {i: r.cpu().numpy() for i, r in c4_recs_d.items()}
        host_versions = {}
        for ver in range(1, self.plan.n_versions):
            vb, vo, _ = versions[ver]
            o = vo.cpu().numpy()
            host_versions[ver] = (vb[: int(o[-1])].cpu().numpy(), o)
        fl = flags.cpu().numpy().view(np.uint32)
        t3 = time.perf_counter()
        return DeviceResult(stage_recs, c4_recs, host_versions, fl,
                            {"h2d": t1 - t0, "kernels": t2 - t1, "d2h": t3 - t2})
