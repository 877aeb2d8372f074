"""Document and outcome types (reference src/data_model.rs:5-34).

JSON encodings follow serde's defaults used by the reference (task / outcome messages):
``TextDocument`` -> ``{"id","content","source","added","created","metadata"}`` with chrono's
``NaiveDate``/``NaiveDateTime`` string forms, and ``ProcessingOutcome`` externally tagged
(``{"Success": {...}}``, ``{"Filtered": {"document": ..., "reason": ...}}``,
``{"Error": {"document": ..., "error_message": ..., "worker_id": ...}}``).
"""
from __future__ import annotations

import dataclasses
import datetime as _dt
import json
from typing import Dict, Optional, Tuple, Union

from .errors import SerializationError


def _fmt_naive_dt(d: _dt.datetime) -> str:
    s = d.strftime("%Y-%m-%dT%H:%M:%S")
    if d.microsecond:
        s += f".{d.microsecond:06d}".rstrip("0")
    return s


def _parse_naive_dt(s: str) -> _dt.datetime:
    return _dt.datetime.fromisoformat(s)


@dataclasses.dataclass
class TextDocument:
    id: str = ""
    content: str = ""
    source: str = ""
    added: Optional[_dt.date] = None
    created: Optional[Tuple[_dt.datetime, _dt.datetime]] = None
    metadata: Dict[str, str] = dataclasses.field(default_factory=dict)

    def to_json_obj(self) -> dict:
        return {
            "id": self.id,
            "content": self.content,
            "source": self.source,
            "added": self.added.isoformat() if self.added else None,
            "created": [_fmt_naive_dt(self.created[0]), _fmt_naive_dt(self.created[1])]
            if self.created
            else None,
            "metadata": dict(self.metadata),
        }

    @classmethod
    def from_json_obj(cls, o: dict) -> "TextDocument":
        try:
            for key in ("id", "content", "source", "metadata"):
                if key not in o:
                    raise ValueError(f"missing field `{key}`")
            md = o["metadata"]
            if not isinstance(md, dict) or not all(
                isinstance(k, str) and isinstance(v, str) for k, v in md.items()
            ):
                raise ValueError("invalid type for `metadata`, expected a map of strings")
            added = _dt.date.fromisoformat(o["added"]) if o.get("added") else None
            created = None
            if o.get("created"):
                a, b = o["created"]
                created = (_parse_naive_dt(a), _parse_naive_dt(b))
            return cls(
                id=str(o["id"]),
                content=str(o["content"]),
                source=str(o["source"]),
                added=added,
                created=created,
                metadata=dict(md),
            )
        except (ValueError, TypeError, KeyError) as e:
            raise SerializationError(e) from e

    def to_json(self) -> bytes:
        return json.dumps(self.to_json_obj(), ensure_ascii=False, separators=(",", ":")).encode()

    @classmethod
    def from_json(cls, data: Union[bytes, str]) -> "TextDocument":
        try:
            o = json.loads(data)
        except (ValueError, UnicodeDecodeError) as e:
            raise SerializationError(e) from e
        if not isinstance(o, dict):
            raise SerializationError(ValueError("expected a JSON object"))
        return cls.from_json_obj(o)


@dataclasses.dataclass
class Success:
    document: TextDocument


@dataclasses.dataclass
class Filtered:
    document: TextDocument
    reason: str


@dataclasses.dataclass
class Error:
    document: TextDocument
    error_message: str
    worker_id: str


ProcessingOutcome = Union[Success, Filtered, Error]


def outcome_to_json(o: ProcessingOutcome) -> bytes:
    if isinstance(o, Success):
        obj = {"Success": o.document.to_json_obj()}
    elif isinstance(o, Filtered):
        obj = {"Filtered": {"document": o.document.to_json_obj(), "reason": o.reason}}
    else:
        obj = {
            "Error": {
                "document": o.document.to_json_obj(),
                "error_message": o.error_message,
                "worker_id": o.worker_id,
            }
        }
    return json.dumps(obj, ensure_ascii=False, separators=(",", ":")).encode()


def outcome_from_json(data: Union[bytes, str]) -> ProcessingOutcome:
    try:
        o = json.loads(data)
    except ValueError as e:
        raise SerializationError(e) from e
    if not isinstance(o, dict) or len(o) != 1:
        raise SerializationError(ValueError("expected an externally tagged outcome"))
    (tag, body), = o.items()
    if tag == "Success":
        return Success(TextDocument.from_json_obj(body))
    if tag == "Filtered":
        return Filtered(TextDocument.from_json_obj(body["document"]), body["reason"])
    if tag == "Error":
        return Error(TextDocument.from_json_obj(body["document"]), body["error_message"], body["worker_id"])
    raise SerializationError(ValueError(f"unknown variant `{tag}`"))
