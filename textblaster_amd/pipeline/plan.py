"""Execution planning: map the YAML step list onto content versions and device stages.

The reference runs every step on every document in YAML order (executor.rs:30-57). Here a
batch of documents flows through *content versions*: version 0 is the input text, and every
C4QualityFilter (the only content-mutating step, c4_filters.rs:258) produces the next version.
All record-producing steps that read the same version form one device *stage* (one analysis
kernel launch computes all of them from one decode + segmentation); C4 steps are their own
device passes. TokenCounter and C4BadWordsFilter run on the host.

First-failure semantics are applied afterwards by the resolver, per document, in YAML order.
"""
from __future__ import annotations

import dataclasses
from typing import List

from ..config.pipeline import PipelineConfig

RECORD_STEPS = ("GopherRepetitionFilter", "GopherQualityFilter", "FineWebQualityFilter", "LanguageDetectionFilter")
HOST_STEPS = ("TokenCounter", "C4BadWordsFilter")


@dataclasses.dataclass
class StepPlan:
    index: int
    type: str
    version_in: int        # content version the step reads
    version_out: int       # version after the step (== version_in unless C4)
    stage: int = -1        # device stage index (record steps)
    c4_pass: int = -1      # device C4 pass index


@dataclasses.dataclass
class ExecPlan:
    steps: List[StepPlan]
    stages: List[List[int]]      # per stage: step indices (all read the same version)
    stage_version: List[int]
    c4_steps: List[int]          # step indices of C4 passes, in order
    n_versions: int

    def describe(self) -> str:
        lines = []
        for s in self.steps:
            where = "host" if s.type in HOST_STEPS else ("c4-pass" if s.c4_pass >= 0 else f"stage{s.stage}")
            lines.append(f"  [{s.index}] {s.type:<24} v{s.version_in}->v{s.version_out}  ({where})")
        return "\n".join(lines)


def build_plan(cfg: PipelineConfig) -> ExecPlan:
    steps: List[StepPlan] = []
    v = 0
    for i, sc in enumerate(cfg.pipeline):
        if sc.type == "C4QualityFilter":
            steps.append(StepPlan(i, sc.type, v, v + 1))
            v += 1
        else:
            steps.append(StepPlan(i, sc.type, v, v))
    stages: List[List[int]] = []
    stage_version: List[int] = []
    for ver in range(v + 1):
        idx = [s.index for s in steps if s.type in RECORD_STEPS and s.version_in == ver]
        # at most 8 steps per stage (device limit): split long runs
        for k in range(0, len(idx), 8):
            chunk = idx[k:k + 8]
            for j in chunk:
                steps[j].stage = len(stages)
            stages.append(chunk)
            stage_version.append(ver)
    c4 = [s.index for s in steps if s.type == "C4QualityFilter"]
    for k, j in enumerate(c4):
        steps[j].c4_pass = k
    return ExecPlan(steps, stages, stage_version, c4, v + 1)
