"""Version comparison helpers (parity: reference utils/versions.py:26-56)."""

from __future__ import annotations

import importlib.metadata
import operator
from typing import Union

from packaging.version import Version, parse

STR_OPERATION_TO_FUNC = {">": operator.gt, ">=": operator.ge, "==": operator.eq, "!=": operator.ne, "<=": operator.le, "<": operator.lt}

torch_version = parse(importlib.metadata.version("torch"))


def compare_versions(library_or_version: Union[str, Version], operation: str, requirement_version: str) -> bool:
    """`compare_versions("torch", ">=", "2.4")` or with an explicit Version."""
    if operation not in STR_OPERATION_TO_FUNC:
        raise ValueError(f"`operation` must be one of {list(STR_OPERATION_TO_FUNC)}, received {operation}")
    if isinstance(library_or_version, str):
        library_or_version = parse(importlib.metadata.version(library_or_version))
    return STR_OPERATION_TO_FUNC[operation](library_or_version, parse(requirement_version))


def is_torch_version(operation: str, version: str) -> bool:
    return compare_versions(torch_version, operation, version)
