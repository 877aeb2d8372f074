"""Device kernels vs. the host emulation of the same algorithms (bit-exact records) and vs. the
ICU oracle (end-to-end decisions). Needs an MI355X."""
import os
import sys

import numpy as np
import pytest

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from adversarial import adversarial_corpus  # noqa: E402

from textblaster_amd import native
from textblaster_amd.config import load_pipeline_config
from textblaster_amd.utils import synth

pytestmark = pytest.mark.gpu

EDGE = ["", "   ", "\n\n", "a", "a\r\nb\r\n", "Hello.\n\n\nHello.\n\nHello.", "x [1] y [2, 3]. z",
        "ΣΑΣ ΣΑΣ.", "İstanbul THE the", "cooKie policy is here.", "lorem IPSUM dolor", "{ curly }",
        "日本語のテキストです。", "mixed 日本 text. Another sentence here.", "- bullet\n- bullet\n• x...",
        "a b a b a b a b a b a b a b", "ab c a bc ab c a bc"]


@pytest.fixture(scope="module")
def corpus():
    # adversarial documents (UAX#29 fuzz pool, constructs across the 64-item chunk boundaries)
    texts = synth.make_corpus(3000, 1024, seed=11) + EDGE + adversarial_corpus()
    rng = np.random.default_rng(7)
    # long documents run one workgroup each (BlockPar kernels): a spread of sizes and languages,
    # plus long C4-heavy text (citations, policy lines, javascript, ellipses)
    langs = ["eng", "dan", "swe", "nob", "nno"]
    texts += [synth.make_doc(rng, langs[k % 5], int(s)) for k, s in enumerate(np.geomspace(4500, 90000, 24))]
    c4ish = ("A line with a citation [1] and another [2, 3] here. Read our privacy policy today.\n"
             "JavaScript must be enabled. Short one...\nThe quick brown fox jumps over the lazy dog.\n") * 200
    texts += [c4ish, c4ish.replace("\n", " ")]
    return texts


@pytest.fixture(scope="module")
def runner_parts(host):
    from textblaster_amd.ops import hiprt

    assert hiprt.device_count() > 0
    from textblaster_amd.models.langid import load_default
    from textblaster_amd.pipeline.device import DeviceRunner
    from textblaster_amd.pipeline.plan import build_plan

    cfg = load_pipeline_config("config/pipeline_config.yaml")
    cfg.pipeline = [s for s in cfg.pipeline if s.type != "TokenCounter"]
    steps = [host.make_step(s.native_dict()) for s in cfg.pipeline]
    plan = build_plan(cfg)
    lid = load_default()
    return cfg, steps, plan, DeviceRunner(steps, plan, "cuda:0", lid), lid


def test_device_records_match_host_emulation(host, corpus, runner_parts):
    cfg, steps, plan, runner, lid = runner_parts
    data, off = synth.pack(corpus)
    res = runner.run(data, off)
    n = len(corpus)
    # documents a gate skipped in a pass (csrc/common/gate.h) have zero records there
    def live(step_i):
        p = runner.pass_of_step[step_i]
        return ~((res.dead != 0) & (res.dead <= p)) if res.dead is not None else np.ones(n, bool)

    for s, idx in enumerate(plan.stages):
        ver = plan.stage_version[s]
        vd, vo = (data, off) if ver == 0 else res.versions[ver]
        ref, rflags = host.emulate_stage(steps, idx, np.ascontiguousarray(vd), np.ascontiguousarray(vo), 8,
                                         lid.native())
        got = res.stage_recs[s]
        width_total, layout = runner.stage_layout[s]
        for (kind, width, prefix), step_i in sorted(zip(layout, idx), key=lambda t: t[0][0] == 4):
            a = got[prefix * n:(prefix + width) * n].reshape(n, width)
            b = ref[prefix * n:(prefix + width) * n].reshape(n, width)
            ok = (res.flags == 0) & (rflags == 0) & live(step_i)
            if kind == 4:
                # language id: exact integer n-gram sums on both sides, so the language is equal;
                # the f64 softmax may differ in the last ulp of exp (device libm vs host)
                ca = a[:, 1].copy().view(np.float64)
                cb = b[:, 1].copy().view(np.float64)
                assert np.array_equal(a[ok, 0], b[ok, 0]), np.nonzero(ok & (a[:, 0] != b[:, 0]))[0][:5]
                assert np.allclose(ca[ok], cb[ok], rtol=0, atol=1e-12)
            else:
                bad = np.nonzero(~np.all(a[ok] == b[ok], axis=1))[0]
                assert len(bad) == 0, (steps[step_i].name, bad[:5], a[ok][bad[:3]], b[ok][bad[:3]])
    # C4 pass: records and rewritten text
    for i in plan.c4_steps:
        ver = plan.steps[i].version_in
        vd, vo = (data, off) if ver == 0 else res.versions[ver]
        rrec, rdata, roff, rflags = host.emulate_c4(steps[i], np.ascontiguousarray(vd), np.ascontiguousarray(vo), 8)
        ok = (res.flags == 0) & (rflags == 0) & live(i)
        assert np.array_equal(res.c4_recs[i].reshape(n, 7)[ok], rrec.reshape(n, 7)[ok])
        gd, go = res.versions[plan.steps[i].version_out]
        for d in np.nonzero(ok)[0]:
            assert bytes(gd[go[d]:go[d + 1]]) == bytes(rdata[roff[d]:roff[d + 1]])


def test_device_gate_matches_host_gate(host, corpus, runner_parts):
    """The gate kernel marks the same documents dead as the host run of the same code over the
    emulated records (language-id near-ties aside), and it does skip work."""
    from textblaster_amd.pipeline.device import EmulatedRunner

    cfg, steps, plan, runner, lid = runner_parts
    data, off = synth.pack(corpus)
    res = runner.run(data, off)
    emu = EmulatedRunner(steps, plan, lid, 8).run(data, off)
    assert res.dead is not None and emu.dead is not None
    assert np.count_nonzero(res.dead) > len(corpus) // 10
    ok = (res.flags == 0) & (emu.flags == 0)
    diff = np.nonzero(ok & (res.dead != emu.dead))[0]
    assert len(diff) <= max(2, len(corpus) // 500), diff[:10]


def test_dictionary_scripts_are_flagged(host, runner_parts, monkeypatch):
    """A dictionary-script document leaves the device only when it reaches a segmentation pass
    without host word marks: the CJK document fails the language gate on the device (exact records,
    not delegated); the Danish document with a CJK snippet passes it and stays on the device with
    the host's ICU marks of its snippet line, or (TB_TUNE dict_marks=0) is flagged by the stage
    kernel's decode."""
    from textblaster_amd.pipeline.device import DeviceRunner

    _, steps, plan, runner, lid = runner_parts
    rng = np.random.default_rng(5)
    dan = synth.make_doc(rng, "dan", 1500)
    data, off = synth.pack(["日本語のテキストです。", "plain english text here.", dan[:200] + " 日本語 " + dan[200:]])
    res = runner.run(data, off)
    assert res.flags[0] == 0 and res.dead[0] != 0
    assert res.flags[1] == 0
    assert res.flags[2] == 0 and runner.dict_marks
    monkeypatch.setenv("TB_TUNE", "dict_marks=0")
    nomarks = DeviceRunner(steps, plan, runner.device, lid)
    res = nomarks.run(data, off)
    assert res.flags[0] == 0 and res.flags[1] == 0
    assert res.flags[2] != 0


def _langid_records(runner, res, n):
    _, layout = runner.stage_layout[0]
    _, w, prefix = [t for t in layout if t[0] == 4][0]
    return res.stage_recs[0][prefix * n:(prefix + w) * n].reshape(n, w)


def _assert_langid_equal(texts, r, m):
    """Device language records == the host model (csrc/common/langid.h): same language and the
    same confidence bits (exact sums / exact MFMA integers, explicit-fma exp on both sides)."""
    bad = []
    for i, t in enumerate(texts):
        lang, conf = m.detect(t)
        got = float(np.frombuffer(np.int64(r[i, 1]).tobytes(), np.float64)[0]) if r[i, 0] >= 0 else 0.0
        if int(r[i, 0]) != lang or got != conf:
            bad.append((i, int(r[i, 0]), lang, got, conf))
    assert not bad, bad[:5]


def test_langid_records_match_host(host, corpus, runner_parts):
    """k_langid_mfma (v3: int8 embedding bag, bf16 MFMA head over 16-document tiles) vs. the host
    model on the corpus: same exact sums and head integers, so the same language and confidence."""
    _, _, _, runner, lid = runner_parts
    assert lid.version == 3 and runner.lid_E is not None
    texts = corpus[:517]  # not a multiple of the 16-document tile
    data, off = synth.pack(texts)
    res = runner.run(data, off)
    _assert_langid_equal(texts, _langid_records(runner, res, len(texts)), lid.native())


def test_langid_mfma_head_vs_fp32_reference(host, corpus, runner_parts):
    """The device's MFMA head vs. plain fp32 inference of the same fastText model in PyTorch
    (mean of the gathered int8 rows in fp32, fp32 head, softmax): logits agree within the
    doc vector's 8-bit quantisation (confidence within 0.015), the argmax is the same away
    from near-ties."""
    import torch

    _, _, _, runner, lid = runner_parts
    h = native.host()
    texts = corpus[:300]
    data, off = synth.pack(texts)
    res = runner.run(data, off)
    r = _langid_records(runner, res, len(texts))
    W = torch.from_numpy(lid.W.reshape(h.LID_DIM, h.LID_LANGS).astype(np.float32)) * float(lid.w_scale)
    b = torch.from_numpy(lid.b[:h.LID_LANGS].astype(np.float32))
    E = torch.from_numpy(lid.E.reshape(h.LID_BUCKETS, h.LID_ROW_DIM).astype(np.float32))
    near = 0
    for i, t in enumerate(texts):
        g, order = h.langid_buckets(t, True)
        if len(g) == 0:
            assert r[i, 0] == -1
            continue
        g = torch.tensor(g, dtype=torch.int64)
        hi = torch.tensor(order) >= 3
        v = torch.cat([E[g[~hi]].sum(0), E[g[hi]].sum(0)]) / len(g)  # the two bags, mean
        logits = v @ W + b
        p = torch.softmax(logits, 0)
        top2 = torch.topk(logits, 2).values
        got = float(np.frombuffer(np.int64(r[i, 1]).tobytes(), np.float64)[0])
        if int(r[i, 0]) != int(torch.argmax(logits)):
            assert float(top2[0] - top2[1]) < 0.05
            near += 1
            continue
        assert abs(got - float(p.max())) < 0.015, (i, got, float(p.max()))
    assert near <= 2


def test_langid_edge_cases_bit_exact(host, runner_parts):
    """The cases the kernel's chunking has to get right: empty and letter-free documents, a word
    cut at the 4096-code-point limit, multibyte letters across 64-byte chunk edges (the 4-gram
    needs three previous letters, found in earlier lanes or in memory), and long documents."""
    rng = np.random.default_rng(7)
    words = ["blåbærgrød", "æblet", "Øresund", "straße", "the", "och", "kærlighed", "ÆØÅ", "naïve", "ab", "x"]
    texts = ["", "1234 5678 !!!", "a", "Å", " \n\n ", "x" * 5000, ("ø" * 4095) + "abc def",
             ("z" * 4094) + " qq", "ab", "abc", "ø ø øø øøø øøøø"]
    for k in (61, 62, 63, 64, 65, 66, 127, 128, 129, 4095, 4096, 4097, 9000):
        t = " ".join(rng.choice(words) for _ in range(k // 4 + 1))
        texts.append(t[:k])
    for shift in range(8):  # multibyte letters straddling the chunk edge at every offset
        texts.append("a" * (60 + shift) + "ææææ øå bcd")
    # the kernel's inline Latin-1 letters (U+00C0..U+00FF, incl. the non-letters × and ÷) and its
    # pair-table alphabet edges: letters outside it (é, ü, ß, Þ, Greek, Cyrillic, CJK) next to ones in it
    latin1 = "".join(chr(c) for c in range(0xC0, 0x100))
    texts += [latin1, " ".join(latin1[i:i + 3] for i in range(0, 64, 3)), "éa aé éé üøß Þorn þá ×÷ ÿ",
              "Ωmega ωα aω Ж жa 中文a aä öü ÅÄÖ", "æ" * 40 + "é" + "ø" * 40, "a\xc3"]
    _, _, _, runner, lid = runner_parts
    data, off = synth.pack(texts)
    res = runner.run(data, off)
    _assert_langid_equal(texts, _langid_records(runner, res, len(texts)), lid.native())


def test_device_run_is_deterministic(host, corpus, runner_parts):
    """Run-twice check: records, flags, gate codes and rewritten texts are
    bitwise identical across runs, whatever the wave scheduling and the LDS atomics order."""
    _, _, plan, runner, _ = runner_parts
    data, off = synth.pack(corpus)
    a = runner.run(data, off)
    b = runner.run(data, off)
    for x, y in zip(a.stage_recs, b.stage_recs):
        np.testing.assert_array_equal(x, y)
    for i in a.c4_recs:
        np.testing.assert_array_equal(a.c4_recs[i], b.c4_recs[i])
    np.testing.assert_array_equal(a.flags, b.flags)
    np.testing.assert_array_equal(a.dead, b.dead)
    for v in a.versions:
        np.testing.assert_array_equal(a.versions[v][0], b.versions[v][0])
        np.testing.assert_array_equal(a.versions[v][1], b.versions[v][1])


def test_split_documents_match_host_emulation(host, corpus, runner_parts, monkeypatch):
    """SURVEY 5.7 intra-document split (k_gr_dup_split: one workgroup per duplicated n-gram order)
    with the split threshold at the long-document threshold, so every workgroup-path document of
    the corpus (4.5-90 KB) is split: GopherRepetition records stay bit-exact against the host."""
    from textblaster_amd.pipeline.device import KIND_GOPHER_REP, DeviceRunner

    cfg, steps, plan, _, lid = runner_parts
    monkeypatch.setenv("TB_TUNE", "split_doc_bytes=1")  # clamped to the long-document threshold
    runner = DeviceRunner(steps, plan, "cuda:0", lid)
    assert runner.gr_split and runner.split_doc_bytes == runner.long_doc_bytes
    data, off = synth.pack(corpus)
    n = len(corpus)
    lens = np.diff(off)
    assert np.count_nonzero(lens > runner.split_doc_bytes) >= 20
    res = runner.run(data, off)
    for s, idx in enumerate(plan.stages):
        if s not in runner.gr_split:
            continue
        ref, rflags = host.emulate_stage(steps, idx, np.ascontiguousarray(data), np.ascontiguousarray(off), 8,
                                         lid.native())
        width_total, layout = runner.stage_layout[s]
        for (kind, width, prefix), step_i in zip(layout, idx):
            if kind != KIND_GOPHER_REP:
                continue
            p = runner.pass_of_step[step_i]
            live = ~((res.dead != 0) & (res.dead <= p)) if res.dead is not None else np.ones(n, bool)
            ok = (res.flags == 0) & (rflags == 0) & live
            assert np.count_nonzero(ok & (lens > runner.split_doc_bytes)) >= 10  # split docs compared
            a = res.stage_recs[s][prefix * n:(prefix + width) * n].reshape(n, width)
            b = ref[prefix * n:(prefix + width) * n].reshape(n, width)
            bad = np.nonzero(~np.all(a[ok] == b[ok], axis=1))[0]
            assert len(bad) == 0, (bad[:5], a[ok][bad[:3]], b[ok][bad[:3]])


def test_pre_decoded_long_documents_match_host(host, runner_parts, monkeypatch):
    """SURVEY 5.7 pre-pass (k_pre_count / k_pre_decode / k_pre_wb): documents of 64 KB and more get
    their code points and word-break marks from many workgroups before their stage workgroup runs.
    Stage records and flags equal the host emulation and a device run without the pre-pass;
    Unicode-heavy text (marks, ZWJ / emoji, regional indicators across 16 KB tile borders) and a
    dictionary-script document (flagged for the CPU path) included."""
    from gpu_fuzz_corpus import fuzz_docs

    from textblaster_amd.pipeline.device import DeviceRunner

    cfg, steps, plan, _, lid = runner_parts
    # (the pre-pass documents take no host word marks: compare both runs with the CPU path for
    # dictionary scripts)
    monkeypatch.setenv("TB_TUNE", "dict_marks=0")
    rng = np.random.default_rng(3)
    langs = ["eng", "dan", "swe", "nob", "nno"]
    texts = [synth.make_doc(rng, langs[k % 5], int(s)) for k, s in enumerate(np.geomspace(66000, 400000, 8))]
    uni = "\n".join(fuzz_docs(3000, seed=9))
    texts += [uni[:150000], uni[150000:230000]]
    # (Danish: it passes the language gate, so it reaches the stage that flags it)
    texts += [synth.make_doc(rng, "dan", 70000) + " 日本語のテキストです。 " + synth.make_doc(rng, "dan", 5000)]
    texts += synth.make_corpus(200, 900, seed=4)  # short documents in the same batch
    data, off = synth.pack(texts)
    n = len(texts)
    lens = np.diff(off)
    res = {}
    for pre in ("65536", "0"):
        monkeypatch.setenv("TB_TUNE", f"dict_marks=0,pre_doc_bytes={pre}")
        runner = DeviceRunner(steps, plan, "cuda:0", lid)
        assert runner.pre_doc_bytes == (65536 if pre != "0" else 0)
        res[pre] = runner.run(data, off)
    a, b = res["65536"], res["0"]
    np.testing.assert_array_equal(a.flags, b.flags)
    assert a.flags[10] != 0  # the dictionary-script document
    for s, idx in enumerate(plan.stages):
        ver = plan.stage_version[s]
        vd, vo = (data, off) if ver == 0 else a.versions[ver]
        np.testing.assert_array_equal(a.stage_recs[s], b.stage_recs[s])
        ref, rflags = host.emulate_stage(steps, idx, np.ascontiguousarray(vd), np.ascontiguousarray(vo), 8,
                                         lid.native())
        for (kind, width, prefix), step_i in zip(runner.stage_layout[s][1], idx):
            if kind == 4:
                continue
            ok = (a.flags == 0) & (rflags == 0)
            if a.dead is not None:
                ok &= ~((a.dead != 0) & (a.dead <= runner.pass_of_step[step_i]))
            if ver == 0:
                assert np.count_nonzero(ok & (lens >= 65536)) >= 2
            x = a.stage_recs[s][prefix * n:(prefix + width) * n].reshape(n, width)
            y = ref[prefix * n:(prefix + width) * n].reshape(n, width)
            bad = np.nonzero(~np.all(x[ok] == y[ok], axis=1))[0]
            assert len(bad) == 0, (steps[step_i].name, bad[:5])
