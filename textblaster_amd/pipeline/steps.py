"""Per-document processing API, mirroring the reference's ``ProcessingStep`` trait and its seven
step implementations (reference executor.rs:8-15, pipeline/filters/*.rs, token_counter.rs).

Each filter computes the same per-document record as the batched engine (C++ host runtime,
``compute_record``) and applies the shared decision/formatting code (``decide``), so reason
strings and metadata are identical on every path. Filtering is signalled by raising
:class:`DocumentFiltered` carrying the (possibly rewritten) document, as in the reference.

Constructor signatures follow the reference's ``new(...)`` functions; parameters are public
attributes that tests may change after construction (the native config is rebuilt lazily).
"""
from __future__ import annotations

import abc
import asyncio
import dataclasses
import os
import struct
from typing import Dict, List, Optional, Sequence, Tuple

from .. import native
from ..config import pipeline as cfgmod
from ..data_model import TextDocument
from ..errors import DocumentFiltered, PipelineError, Unexpected


class ProcessingStep(abc.ABC):
    """A pipeline step: ``process`` returns the (possibly modified) document or raises
    :class:`DocumentFiltered` / another :class:`PipelineError`."""

    @abc.abstractmethod
    def name(self) -> str: ...

    @abc.abstractmethod
    def process(self, document: TextDocument) -> TextDocument: ...

    async def process_async(self, document: TextDocument) -> TextDocument:
        return self.process(document)


def _apply_meta(doc: TextDocument, meta: Sequence[Tuple[str, str]]) -> None:
    for k, v in meta:
        doc.metadata[k] = v


class _NativeStep(ProcessingStep):
    TYPE = ""
    _FIELDS: Tuple[str, ...] = ()

    def __init__(self, segmentation: str = "icu"):
        self.segmentation = segmentation
        self._cache_key = None
        self._native = None

    def _params_dict(self) -> Dict:
        d = {"type": self.TYPE}
        for f in self._FIELDS:
            d[f] = getattr(self, f)
        return d

    def native_step(self):
        d = self._params_dict()
        key = repr(sorted(d.items(), key=lambda kv: kv[0]))
        if key != self._cache_key:
            self._native = native.host().make_step(d)
            self._cache_key = key
        return self._native

    def name(self) -> str:
        return self.TYPE

    def _record(self, doc: TextDocument):
        rec, new = native.host().compute_record(self.native_step(), doc.content, self.segmentation)
        return list(rec), new

    def process(self, document: TextDocument) -> TextDocument:
        h = native.host()
        rec, new = self._record(document)
        passed, error, reason, meta = h.decide(self.native_step(), rec)
        self._post(document, rec, new)
        _apply_meta(document, meta)
        if error:
            raise Unexpected(reason)
        if not passed:
            raise DocumentFiltered(document, reason)
        return document

    def _post(self, doc, rec, new) -> None:
        pass


class C4QualityFilter(_NativeStep):
    """reference c4_filters.rs:72-295"""

    TYPE = "C4QualityFilter"
    _FIELDS = ("split_paragraph", "remove_citations", "filter_no_terminal_punct", "min_num_sentences",
               "min_words_per_line", "max_word_length", "filter_lorem_ipsum", "filter_javascript",
               "filter_curly_bracket", "filter_policy")

    def __init__(self, split_paragraph: bool, remove_citations: bool, filter_no_terminal_punct: bool,
                 min_num_sentences: int, min_words_per_line: int, max_word_length: int,
                 filter_lorem_ipsum: bool, filter_javascript: bool, filter_curly_bracket: bool,
                 filter_policy: bool, segmentation: str = "icu"):
        super().__init__(segmentation)
        self.split_paragraph = split_paragraph
        self.remove_citations = remove_citations
        self.filter_no_terminal_punct = filter_no_terminal_punct
        self.min_num_sentences = min_num_sentences
        self.min_words_per_line = min_words_per_line
        self.max_word_length = max_word_length
        self.filter_lorem_ipsum = filter_lorem_ipsum
        self.filter_javascript = filter_javascript
        self.filter_curly_bracket = filter_curly_bracket
        self.filter_policy = filter_policy

    def _post(self, doc, rec, new) -> None:
        if not rec[0] and not rec[1]:  # no lorem/curly early exit: content is rewritten
            doc.content = new.decode("utf-8")


class GopherRepetitionFilter(_NativeStep):
    """reference gopher_rep.rs:12-220"""

    TYPE = "GopherRepetitionFilter"
    _FIELDS = ("dup_line_frac", "dup_para_frac", "dup_line_char_frac", "dup_para_char_frac", "top_n_grams",
               "dup_n_grams")

    def __init__(self, dup_line_frac=None, dup_para_frac=None, dup_line_char_frac=None, dup_para_char_frac=None,
                 top_n_grams=(), dup_n_grams=(), segmentation: str = "icu"):
        super().__init__(segmentation)
        self.dup_line_frac = dup_line_frac
        self.dup_para_frac = dup_para_frac
        self.dup_line_char_frac = dup_line_char_frac
        self.dup_para_char_frac = dup_para_char_frac
        self.top_n_grams = list(top_n_grams)
        self.dup_n_grams = list(dup_n_grams)


class GopherQualityFilter(_NativeStep):
    """reference gopher_quality.rs:19-318"""

    TYPE = "GopherQualityFilter"
    _FIELDS = ("min_doc_words", "max_doc_words", "min_avg_word_length", "max_avg_word_length",
               "max_symbol_word_ratio", "max_bullet_lines_ratio", "max_ellipsis_lines_ratio",
               "max_non_alpha_words_ratio", "min_stop_words", "stop_words")

    def __init__(self, min_doc_words=None, max_doc_words=None, min_avg_word_length=None,
                 max_avg_word_length=None, max_symbol_word_ratio=None, max_bullet_lines_ratio=None,
                 max_ellipsis_lines_ratio=None, max_non_alpha_words_ratio=None, min_stop_words=None,
                 stop_words: Optional[List[str]] = None, segmentation: str = "icu"):
        super().__init__(segmentation)
        self.min_doc_words = min_doc_words
        self.max_doc_words = max_doc_words
        self.min_avg_word_length = min_avg_word_length
        self.max_avg_word_length = max_avg_word_length
        self.max_symbol_word_ratio = max_symbol_word_ratio
        self.max_bullet_lines_ratio = max_bullet_lines_ratio
        self.max_ellipsis_lines_ratio = max_ellipsis_lines_ratio
        self.max_non_alpha_words_ratio = max_non_alpha_words_ratio
        self.min_stop_words = min_stop_words
        self.stop_words = list(stop_words) if stop_words is not None else list(cfgmod.DEFAULT_STOP_WORDS)


class FineWebQualityFilter(_NativeStep):
    """reference fineweb_quality.rs:29-226"""

    TYPE = "FineWebQualityFilter"
    _FIELDS = ("line_punct_thr", "line_punct_exclude_zero", "short_line_thr", "short_line_length",
               "char_duplicates_ratio", "new_line_ratio")

    def __init__(self, line_punct_thr: float, line_punct_exclude_zero: bool, short_line_thr: float,
                 short_line_length: int, char_duplicates_ratio: float, new_line_ratio: float,
                 stop_chars: Optional[Sequence[str]] = None, segmentation: str = "icu"):
        super().__init__(segmentation)
        self.line_punct_thr = line_punct_thr
        self.line_punct_exclude_zero = line_punct_exclude_zero
        self.short_line_thr = short_line_thr
        self.short_line_length = short_line_length
        self.char_duplicates_ratio = char_duplicates_ratio
        self.new_line_ratio = new_line_ratio
        self.stop_chars = set(stop_chars) if stop_chars is not None else set(cfgmod.DEFAULT_STOP_CHARS)

    def _params_dict(self) -> Dict:
        d = super()._params_dict()
        d["stop_chars"] = sorted(ord(c) for c in self.stop_chars)
        return d


class LanguageDetectionFilter(ProcessingStep):
    """reference language_filter.rs:7-93 (fastText-style model instead of lingua, see models.langid)"""

    def __init__(self, min_confidence: float, allowed_langs: Sequence[str], model=None):
        from ..models.langid import load_default

        self.min_confidence = min_confidence
        self.allowed_langs = list(allowed_langs)
        self.model = model or load_default()

    def name(self) -> str:
        return "LanguageDetectionFilter"

    def native_step(self):
        sc = cfgmod.StepConfig("LanguageDetectionFilter",
                               cfgmod.LanguageDetectionParams(self.min_confidence, self.allowed_langs))
        return native.host().make_step(sc.native_dict())

    def process(self, document: TextDocument) -> TextDocument:
        h = native.host()
        lang, conf = self.model.native().detect(document.content)
        rec = [lang, struct.unpack("<q", struct.pack("<d", conf))[0]]
        passed, _, reason, meta = h.decide(self.native_step(), rec)
        _apply_meta(document, meta)
        if not passed:
            raise DocumentFiltered(document, reason)
        return document


class TokenCounter(ProcessingStep):
    """reference token_counter.rs:8-43; ``tokenizer_name`` is resolved locally (no network)."""

    def __init__(self, tokenizer_name: str, tokenizer_dir: Optional[str] = None):
        from ..models.tokenizer import load_tokenizer

        self.tokenizer = load_tokenizer(tokenizer_name, tokenizer_dir)

    def name(self) -> str:
        return "TokenCounter"

    def process(self, document: TextDocument) -> TextDocument:
        try:
            n = self.tokenizer.count([document.content])[0]
        except Exception as e:  # noqa: BLE001
            raise Unexpected(str(e)) from e
        document.metadata["token_count"] = str(n)
        return document


class C4BadWordsFilter(ProcessingStep):
    """reference c4_filters.rs:298-551. Word lists are read from ``cache_base_path`` (or
    ``data/c4_badwords``); nothing is downloaded. The keep-fraction draws come from a rand-0.8
    compatible ``StdRng`` stream seeded like the reference."""

    CJK = ("ja", "th", "zh")

    def __init__(self, params: cfgmod.C4BadWordsParams):
        import random

        self.params = params
        h = native.host()
        self.module = h.BadWordsModule(params.cache_base_path or os.path.join("data", "c4_badwords"))
        seed = params.seed if params.seed is not None else random.getrandbits(64)
        self.rng = h.StdRng(seed)

    def name(self) -> str:
        return "C4BadWordsFilter"

    def process(self, document: TextDocument) -> TextDocument:
        lang = document.metadata.get("language", self.params.default_language)
        try:
            supported, has_list = self.module.lookup(lang)
        except RuntimeError as e:
            reason = f"I/O error: {e}"
            document.metadata["c4_badwords_filter_status"] = "filtered"
            document.metadata["c4_badwords_filter_reason"] = reason
            raise DocumentFiltered(document, reason) from e
        if not supported:
            if self.params.fail_on_missing_language:
                reason = (f"There is no badwords list available for '{lang}'. "
                          f"Set fail_on_missing_language=False to continue anyway.")
                document.metadata["c4_badwords_filter_status"] = "filtered"
                document.metadata["c4_badwords_filter_reason"] = reason
                raise DocumentFiltered(document, reason)
            document.metadata["c4_badwords_filter_status"] = "passed_no_regex"
            return document
        if not has_list:
            document.metadata["c4_badwords_filter_status"] = "passed_no_regex"
            return document
        if self.module.matches(lang, document.content):
            if self.params.keep_fraction > 0.0 and self.rng.gen_f32() < self.params.keep_fraction:
                document.metadata["c4_badwords_filter_status"] = "passed_kept_by_fraction"
                return document
            reason = "document_removed_with_badwords"
            document.metadata["c4_badwords_filter_status"] = "filtered"
            document.metadata["c4_badwords_filter_reason"] = reason
            raise DocumentFiltered(document, reason)
        document.metadata["c4_badwords_filter_status"] = "passed"
        return document


def step_from_config(sc: cfgmod.StepConfig, tokenizer_dir: Optional[str] = None,
                     segmentation: str = "icu") -> ProcessingStep:
    p = sc.params
    t = sc.type
    if t == "C4QualityFilter":
        return C4QualityFilter(p.split_paragraph, p.remove_citations, p.filter_no_terminal_punct,
                               p.min_num_sentences, p.min_words_per_line, p.max_word_length,
                               p.filter_lorem_ipsum, p.filter_javascript, p.filter_curly_bracket,
                               p.filter_policy, segmentation=segmentation)
    if t == "GopherRepetitionFilter":
        return GopherRepetitionFilter(p.dup_line_frac, p.dup_para_frac, p.dup_line_char_frac,
                                      p.dup_para_char_frac, p.top_n_grams, p.dup_n_grams, segmentation=segmentation)
    if t == "GopherQualityFilter":
        return GopherQualityFilter(p.min_doc_words, p.max_doc_words, p.min_avg_word_length,
                                   p.max_avg_word_length, p.max_symbol_word_ratio, p.max_bullet_lines_ratio,
                                   p.max_ellipsis_lines_ratio, p.max_non_alpha_words_ratio, p.min_stop_words,
                                   p.stop_words, segmentation=segmentation)
    if t == "FineWebQualityFilter":
        return FineWebQualityFilter(p.line_punct_thr, p.line_punct_exclude_zero, p.short_line_thr,
                                    p.short_line_length, p.char_duplicates_ratio, p.new_line_ratio,
                                    p.stop_chars, segmentation=segmentation)
    if t == "LanguageDetectionFilter":
        return LanguageDetectionFilter(p.min_confidence, p.allowed_languages)
    if t == "TokenCounter":
        return TokenCounter(p.tokenizer_name, tokenizer_dir)
    if t == "C4BadWordsFilter":
        return C4BadWordsFilter(p)
    raise Unexpected(f"unknown step type {t}")
