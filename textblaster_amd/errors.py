"""Error model (reference src/error.rs:6-61).

Filtering is signalled with :class:`DocumentFiltered` on the per-document API, exactly like the
reference; the batched engine carries the same information as data (fail step + reason).
"""
from __future__ import annotations


class PipelineError(Exception):
    """Base class of every pipeline error."""


class ConfigError(PipelineError):
    def __init__(self, msg: str):
        super().__init__(msg)
        self.msg = msg

    def __str__(self) -> str:
        return f"Configuration error: {self.msg}"


class IoError(PipelineError):
    def __init__(self, source: BaseException):
        super().__init__(str(source))
        self.source = source

    def __str__(self) -> str:
        return f"I/O error: {self.source}"


class ParquetError(PipelineError):
    def __init__(self, source):
        super().__init__(str(source))
        self.source = source

    def __str__(self) -> str:
        return f"Parquet reading error: {self.source}"


class ArrowError(PipelineError):
    def __init__(self, source):
        super().__init__(str(source))
        self.source = source

    def __str__(self) -> str:
        return f"Arrow conversion error: {self.source}"


class DocumentFiltered(PipelineError):
    def __init__(self, document, reason: str):
        super().__init__(reason)
        self.document = document
        self.reason = reason

    def __str__(self) -> str:
        return f"Document '{self.document.id}' filtered out: {self.reason}"


class StepError(PipelineError):
    def __init__(self, step_name: str, source: PipelineError):
        super().__init__(step_name)
        self.step_name = step_name
        self.source = source

    def __str__(self) -> str:
        return f"Error in processing step '{self.step_name}': {self.source}"


class QueueError(PipelineError):
    def __init__(self, msg: str):
        super().__init__(msg)
        self.msg = msg

    def __str__(self) -> str:
        return f"Queueing system error: {self.msg}"


class SerializationError(PipelineError):
    def __init__(self, source):
        super().__init__(str(source))
        self.source = source

    def __str__(self) -> str:
        return f"Serialization/Deserialization error: {self.source}"


class ConfigValidationError(PipelineError):
    def __init__(self, msg: str):
        super().__init__(msg)
        self.msg = msg

    def __str__(self) -> str:
        return f"Configuration validation error: {self.msg}"


class Unexpected(PipelineError):
    def __init__(self, msg: str):
        super().__init__(msg)
        self.msg = msg

    def __str__(self) -> str:
        return f"Unexpected error: {self.msg}"


class DeviceError(PipelineError):
    """A HIP/RCCL failure on the device path (new in this framework)."""

    def __init__(self, msg: str):
        super().__init__(msg)
        self.msg = msg

    def __str__(self) -> str:
        return f"Device error: {self.msg}"
