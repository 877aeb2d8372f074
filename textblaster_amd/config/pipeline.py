"""Pipeline configuration: the reference's ``pipeline_config.yaml`` schema, parsing rules and
validation messages (reference src/config/pipeline.rs:10-393, survey Appendix B).

The YAML layout is ``pipeline: [ {type: <StepName>, <flattened params>...}, ... ]`` (serde
internally-tagged enum). Unknown keys are ignored, missing required keys are errors
(``missing field `x```), ``Option`` keys may be omitted, list keys default to empty.
"""
from __future__ import annotations

import dataclasses
import math
import os
from typing import Any, Dict, List, Optional, Sequence, Tuple, Union

import numpy as np
import yaml

from ..errors import ConfigError, ConfigValidationError

STEP_TYPES = (
    "C4QualityFilter",
    "GopherRepetitionFilter",
    "GopherQualityFilter",
    "C4BadWordsFilter",
    "LanguageDetectionFilter",
    "FineWebQualityFilter",
    "TokenCounter",
)

# reference gopher_quality.rs:10
DEFAULT_STOP_WORDS = ["the", "be", "to", "of", "and", "that", "have", "with"]
# reference fineweb_quality.rs:26 END_PUNCTUATION
DEFAULT_STOP_CHARS = [".", "!", "?", '"', "'", "”"]

# ISO 639-3 codes known to lingua 1.7 (IsoCode639_3::try_from accepts exactly these).
LINGUA_ISO_639_3 = (
    "afr sqi ara hye aze eus bel ben nob bos bul cat zho hrv ces dan nld eng epo est fin fra lug kat "
    "deu ell guj heb hin hun isl ind gle ita jpn kaz kor lat lav lit mkd msa mri mar mon nno fas pol "
    "por pan ron rus srp sna slk slv som sot spa swa swe tgl tam tel tha tso tsn tur ukr urd vie cym "
    "xho yor zul"
).split()
# Candidate languages of the detector (reference language_filter.rs:39-45), in model order.
LANG_CODES = ("eng", "dan", "swe", "nno", "nob")
LANG_NAMES = ("English", "Danish", "Swedish", "Nynorsk", "Bokmal")


def rust_f64(x: float) -> str:
    """Rust ``f64`` Display: shortest round-trip digits, never exponent notation."""
    if math.isnan(x):
        return "NaN"
    if math.isinf(x):
        return "inf" if x > 0 else "-inf"
    return np.format_float_positional(float(x), unique=True, trim="-")


def rust_f32(x: float) -> str:
    return np.format_float_positional(np.float32(x), unique=True, trim="-")


# --------------------------------------------------------------------------------------------
# serde-like field decoding

class _SerdeError(Exception):
    pass


def _type_name(v: Any) -> str:
    if isinstance(v, bool):
        return f"boolean `{str(v).lower()}`"
    if isinstance(v, int):
        return f"integer `{v}`"
    if isinstance(v, float):
        return f"floating point `{rust_f64(v)}`"
    if isinstance(v, str):
        return f"string {v!r}"
    if isinstance(v, list):
        return "sequence"
    if isinstance(v, dict):
        return "map"
    if v is None:
        return "unit value"
    return type(v).__name__


def _as_bool(v, name):
    if isinstance(v, bool):
        return v
    raise _SerdeError(f"{name}: invalid type: {_type_name(v)}, expected a boolean")


def _as_usize(v, name):
    if isinstance(v, bool) or not isinstance(v, int):
        raise _SerdeError(f"{name}: invalid type: {_type_name(v)}, expected usize")
    if v < 0 or v >= 2**64:
        raise _SerdeError(f"{name}: invalid value: integer `{v}`, expected usize")
    return int(v)


def _as_u64(v, name):
    return _as_usize(v, name)


def _as_f64(v, name):
    if isinstance(v, bool) or not isinstance(v, (int, float)):
        raise _SerdeError(f"{name}: invalid type: {_type_name(v)}, expected f64")
    return float(v)


def _as_f32(v, name):
    return float(np.float32(_as_f64(v, name).__float__()))


def _as_str(v, name):
    if not isinstance(v, str):
        raise _SerdeError(f"{name}: invalid type: {_type_name(v)}, expected a string")
    return v


def _as_char(v, name):
    s = _as_str(v, name)
    if len(s) != 1:
        raise _SerdeError(f"{name}: invalid value: string {s!r}, expected a character")
    return s


def _as_list(v, name, item):
    if not isinstance(v, list):
        raise _SerdeError(f"{name}: invalid type: {_type_name(v)}, expected a sequence")
    return [item(x, name) for x in v]


def _as_ngram_list(v, name):
    def pair(x, nm):
        if not isinstance(x, list) or len(x) != 2:
            raise _SerdeError(f"{nm}: invalid type: {_type_name(x)}, expected a tuple of size 2")
        return (_as_usize(x[0], nm), _as_f64(x[1], nm))

    return _as_list(v, name, pair)


_REQ = object()


@dataclasses.dataclass
class C4QualityParams:
    split_paragraph: bool
    remove_citations: bool
    filter_no_terminal_punct: bool
    min_num_sentences: int
    min_words_per_line: int
    max_word_length: int
    filter_lorem_ipsum: bool
    filter_javascript: bool
    filter_curly_bracket: bool
    filter_policy: bool

    _fields = (
        ("split_paragraph", _as_bool, _REQ), ("remove_citations", _as_bool, _REQ),
        ("filter_no_terminal_punct", _as_bool, _REQ), ("min_num_sentences", _as_usize, _REQ),
        ("min_words_per_line", _as_usize, _REQ), ("max_word_length", _as_usize, _REQ),
        ("filter_lorem_ipsum", _as_bool, _REQ), ("filter_javascript", _as_bool, _REQ),
        ("filter_curly_bracket", _as_bool, _REQ), ("filter_policy", _as_bool, _REQ),
    )

    def validate(self) -> None:
        for f in ("min_num_sentences", "min_words_per_line", "max_word_length"):
            if getattr(self, f) == 0:
                raise ConfigValidationError(f"C4QualityParams: {f} must be greater than 0")


@dataclasses.dataclass
class GopherRepetitionParams:
    dup_line_frac: Optional[float] = None
    dup_para_frac: Optional[float] = None
    dup_line_char_frac: Optional[float] = None
    dup_para_char_frac: Optional[float] = None
    top_n_grams: List[Tuple[int, float]] = dataclasses.field(default_factory=list)
    dup_n_grams: List[Tuple[int, float]] = dataclasses.field(default_factory=list)

    _fields = (
        ("dup_line_frac", _as_f64, None), ("dup_para_frac", _as_f64, None),
        ("dup_line_char_frac", _as_f64, None), ("dup_para_char_frac", _as_f64, None),
        ("top_n_grams", _as_ngram_list, list), ("dup_n_grams", _as_ngram_list, list),
    )

    def validate(self) -> None:
        for name in ("dup_line_frac", "dup_para_frac", "dup_line_char_frac", "dup_para_char_frac"):
            v = getattr(self, name)
            if v is not None and not (0.0 <= v <= 1.0):
                raise ConfigValidationError(
                    f"GopherRepetitionParams: {name} must be between 0.0 and 1.0, got {rust_f64(v)}")
        for name in ("top_n_grams", "dup_n_grams"):
            for idx, (size, frac) in enumerate(getattr(self, name)):
                if size == 0:
                    raise ConfigValidationError(
                        f"GopherRepetitionParams: n-gram size in {name} at index {idx} must be greater than 0")
                if not (0.0 <= frac <= 1.0):
                    raise ConfigValidationError(
                        f"GopherRepetitionParams: n-gram fraction in {name} at index {idx} must be between "
                        f"0.0 and 1.0, got {rust_f64(frac)}")


@dataclasses.dataclass
class GopherQualityParams:
    min_doc_words: Optional[int] = None
    max_doc_words: Optional[int] = None
    min_avg_word_length: Optional[float] = None
    max_avg_word_length: Optional[float] = None
    max_symbol_word_ratio: Optional[float] = None
    max_bullet_lines_ratio: Optional[float] = None
    max_ellipsis_lines_ratio: Optional[float] = None
    max_non_alpha_words_ratio: Optional[float] = None
    min_stop_words: Optional[int] = None
    stop_words: Optional[List[str]] = None

    _fields = (
        ("min_doc_words", _as_usize, None), ("max_doc_words", _as_usize, None),
        ("min_avg_word_length", _as_f64, None), ("max_avg_word_length", _as_f64, None),
        ("max_symbol_word_ratio", _as_f64, None), ("max_bullet_lines_ratio", _as_f64, None),
        ("max_ellipsis_lines_ratio", _as_f64, None), ("max_non_alpha_words_ratio", _as_f64, None),
        ("min_stop_words", _as_usize, None),
        ("stop_words", lambda v, n: _as_list(v, n, _as_str), None),
    )

    def validate(self) -> None:
        if self.min_doc_words is not None and self.min_doc_words == 0:
            raise ConfigValidationError("GopherQualityParams: min_doc_words must be greater than 0")
        if self.max_doc_words is not None and self.max_doc_words == 0:
            raise ConfigValidationError("GopherQualityParams: max_doc_words must be greater than 0")
        if self.min_doc_words is not None and self.max_doc_words is not None and self.min_doc_words > self.max_doc_words:
            raise ConfigValidationError(
                f"GopherQualityParams: min_doc_words ({self.min_doc_words}) cannot be greater than "
                f"max_doc_words ({self.max_doc_words})")
        if self.min_avg_word_length is not None and self.min_avg_word_length <= 0.0:
            raise ConfigValidationError("GopherQualityParams: min_avg_word_length must be greater than 0.0")
        if self.max_avg_word_length is not None and self.max_avg_word_length <= 0.0:
            raise ConfigValidationError("GopherQualityParams: max_avg_word_length must be greater than 0.0")
        if (self.min_avg_word_length is not None and self.max_avg_word_length is not None
                and self.min_avg_word_length > self.max_avg_word_length):
            raise ConfigValidationError(
                f"GopherQualityParams: min_avg_word_length ({rust_f64(self.min_avg_word_length)}) cannot be "
                f"greater than max_avg_word_length ({rust_f64(self.max_avg_word_length)})")
        for name in ("max_symbol_word_ratio", "max_bullet_lines_ratio", "max_ellipsis_lines_ratio",
                     "max_non_alpha_words_ratio"):
            v = getattr(self, name)
            if v is not None and v < 0.0:
                raise ConfigValidationError(f"GopherQualityParams: {name} must be non-negative, got {rust_f64(v)}")


@dataclasses.dataclass
class C4BadWordsParams:
    keep_fraction: float
    fail_on_missing_language: bool
    default_language: str
    seed: Optional[int] = None
    cache_base_path: Optional[str] = None  # not deserialized (serde(skip)); set by tests / CLI

    _fields = (
        ("keep_fraction", _as_f32, _REQ), ("fail_on_missing_language", _as_bool, _REQ),
        ("seed", _as_u64, None), ("default_language", _as_str, _REQ),
    )

    def validate(self) -> None:
        if not (0.0 <= self.keep_fraction <= 1.0):
            raise ConfigValidationError(
                f"C4BadWordsParams: keep_fraction must be between 0.0 and 1.0, got {rust_f32(self.keep_fraction)}")
        if self.default_language == "":
            raise ConfigValidationError("C4BadWordsParams: default_language cannot be empty")


@dataclasses.dataclass
class LanguageDetectionParams:
    min_confidence: float
    allowed_languages: List[str]

    _fields = (("min_confidence", _as_f64, _REQ),
               ("allowed_languages", lambda v, n: _as_list(v, n, _as_str), _REQ))

    def validate(self) -> None:
        if not (0.0 <= self.min_confidence <= 1.0):
            raise ConfigValidationError(
                f"LanguageDetectionParams: min_confidence must be between 0.0 and 1.0, got {rust_f64(self.min_confidence)}")
        if not self.allowed_languages:
            raise ConfigValidationError("LanguageDetectionParams: allowed_languages cannot be empty")


@dataclasses.dataclass
class FineWebQualityFilterParams:
    line_punct_thr: float
    line_punct_exclude_zero: bool
    short_line_thr: float
    short_line_length: int
    char_duplicates_ratio: float
    new_line_ratio: float
    stop_chars: Optional[List[str]] = None

    _fields = (
        ("line_punct_thr", _as_f64, _REQ), ("line_punct_exclude_zero", _as_bool, _REQ),
        ("stop_chars", lambda v, n: sorted(set(_as_list(v, n, _as_char))), None),
        ("short_line_thr", _as_f64, _REQ), ("short_line_length", _as_usize, _REQ),
        ("char_duplicates_ratio", _as_f64, _REQ), ("new_line_ratio", _as_f64, _REQ),
    )

    def validate(self) -> None:
        for name in ("line_punct_thr", "short_line_thr", "char_duplicates_ratio", "new_line_ratio"):
            v = getattr(self, name)
            if not (0.0 <= v <= 1.0):
                raise ConfigValidationError(
                    f"FineWebQualityFilterParams: {name} must be between 0.0 and 1.0, got {rust_f64(v)}")
        if self.short_line_length == 0:
            raise ConfigValidationError("FineWebQualityFilterParams: short_line_length must be greater than 0")


@dataclasses.dataclass
class TokenCounterParams:
    tokenizer_name: str

    _fields = (("tokenizer_name", _as_str, _REQ),)

    def validate(self) -> None:
        if self.tokenizer_name == "":
            raise ConfigValidationError("TokenCounterParams: tokenizer_name cannot be empty")


PARAMS_BY_TYPE = {
    "C4QualityFilter": C4QualityParams,
    "GopherRepetitionFilter": GopherRepetitionParams,
    "GopherQualityFilter": GopherQualityParams,
    "C4BadWordsFilter": C4BadWordsParams,
    "LanguageDetectionFilter": LanguageDetectionParams,
    "FineWebQualityFilter": FineWebQualityFilterParams,
    "TokenCounter": TokenCounterParams,
}

ParamsT = Union[C4QualityParams, GopherRepetitionParams, GopherQualityParams, C4BadWordsParams,
                LanguageDetectionParams, FineWebQualityFilterParams, TokenCounterParams]


@dataclasses.dataclass
class StepConfig:
    type: str
    params: ParamsT

    def name(self) -> str:
        return self.type

    def validate(self) -> None:
        self.params.validate()

    def native_dict(self) -> Dict[str, Any]:
        """Fully-defaulted parameter dict consumed by the native runtime (``_tbhost.make_step``)."""
        d: Dict[str, Any] = {"type": self.type}
        p = self.params
        for f in dataclasses.fields(p):
            d[f.name] = getattr(p, f.name)
        if self.type == "GopherQualityFilter":
            d["stop_words"] = list(p.stop_words) if p.stop_words is not None else list(DEFAULT_STOP_WORDS)
        elif self.type == "FineWebQualityFilter":
            chars = p.stop_chars if p.stop_chars is not None else DEFAULT_STOP_CHARS
            d["stop_chars"] = [ord(c) for c in chars]
        elif self.type == "LanguageDetectionFilter":
            valid = [c.lower() for c in p.allowed_languages if c.lower() in LINGUA_ISO_639_3]
            d["allowed_codes"] = valid
            d["allowed_langs"] = sorted({LANG_CODES.index(c) for c in valid if c in LANG_CODES})
        return d


@dataclasses.dataclass
class PipelineConfig:
    pipeline: List[StepConfig]

    def validate(self) -> None:
        for s in self.pipeline:
            s.validate()


def _decode_params(cls, raw: dict, where: str):
    kwargs = {}
    for name, conv, default in cls._fields:
        if name in raw and raw[name] is not None:
            kwargs[name] = conv(raw[name], f"{where}.{name}")
        elif name in raw and raw[name] is None and default is _REQ:
            raise _SerdeError(f"{where}: invalid type: unit value, expected {name}")
        elif default is _REQ:
            raise _SerdeError(f"{where}: missing field `{name}`")
        elif default is list:
            kwargs[name] = []
        else:
            kwargs[name] = None
    return cls(**kwargs)


def parse_pipeline_config(obj: Any) -> PipelineConfig:
    """Decode an already-loaded YAML document (raises _SerdeError with serde-like messages)."""
    if not isinstance(obj, dict):
        raise _SerdeError(f"invalid type: {_type_name(obj)}, expected struct PipelineConfig")
    if "pipeline" not in obj:
        raise _SerdeError("missing field `pipeline`")
    steps_raw = obj["pipeline"]
    if not isinstance(steps_raw, list):
        raise _SerdeError(f"pipeline: invalid type: {_type_name(steps_raw)}, expected a sequence")
    steps = []
    for i, raw in enumerate(steps_raw):
        where = f"pipeline[{i}]"
        if not isinstance(raw, dict):
            raise _SerdeError(f"{where}: invalid type: {_type_name(raw)}, expected internally tagged enum StepConfig")
        if "type" not in raw:
            raise _SerdeError(f"{where}: missing field `type`")
        t = raw["type"]
        if t not in PARAMS_BY_TYPE:
            expected = ", ".join(f"`{x}`" for x in STEP_TYPES)
            raise _SerdeError(f"{where}: unknown variant `{t}`, expected one of {expected}")
        steps.append(StepConfig(t, _decode_params(PARAMS_BY_TYPE[t], raw, where)))
    return PipelineConfig(steps)


def load_pipeline_config_str(text: str, path_display: str = "<string>") -> PipelineConfig:
    try:
        obj = yaml.safe_load(text)
        cfg = parse_pipeline_config(obj)
    except (yaml.YAMLError, _SerdeError) as e:
        raise ConfigError(f"Failed to parse pipeline config YAML from '{path_display}': {e}") from e
    cfg.validate()
    return cfg


def load_pipeline_config(path: Union[str, os.PathLike]) -> PipelineConfig:
    """Read + parse + validate (reference config/pipeline.rs:372-393)."""
    p = os.fspath(path)
    try:
        with open(p, "r", encoding="utf-8") as f:
            text = f.read()
    except OSError as e:
        raise ConfigError(f"Failed to read pipeline config file '{p}': {e}") from e
    return load_pipeline_config_str(text, p)
