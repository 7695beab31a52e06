"""Tiny assertion helpers (reference: common/determined_common/check.py:30-321).

Each raises ``CheckFailedError`` with the caller's message, used for user-facing API misuse
errors (the controller turns them into trial errors).
"""
from typing import Any, Container, Optional


class CheckFailedError(Exception):
    pass


def _fail(reason: Optional[str], default: str) -> None:
    raise CheckFailedError(f"{default}: {reason}" if reason else default)


def true(val: Any, reason: Optional[str] = None) -> None:
    if not val:
        _fail(reason, "Check failed: expected true")


def false(val: Any, reason: Optional[str] = None) -> None:
    if val:
        _fail(reason, "Check failed: expected false")


def eq(a: Any, b: Any, reason: Optional[str] = None) -> None:
    if a != b:
        _fail(reason, f"{a!r} != {b!r}")


def not_eq(a: Any, b: Any, reason: Optional[str] = None) -> None:
    if a == b:
        _fail(reason, f"{a!r} == {b!r}")


def gt(a: Any, b: Any, reason: Optional[str] = None) -> None:
    if not a > b:
        _fail(reason, f"{a!r} <= {b!r}")


def gt_eq(a: Any, b: Any, reason: Optional[str] = None) -> None:
    if not a >= b:
        _fail(reason, f"{a!r} < {b!r}")


def lt(a: Any, b: Any, reason: Optional[str] = None) -> None:
    if not a < b:
        _fail(reason, f"{a!r} >= {b!r}")


def lt_eq(a: Any, b: Any, reason: Optional[str] = None) -> None:
    if not a <= b:
        _fail(reason, f"{a!r} > {b!r}")


def is_in(a: Any, container: Container, reason: Optional[str] = None) -> None:
    if a not in container:
        _fail(reason, f"{a!r} not in container")


def not_in(a: Any, container: Container, reason: Optional[str] = None) -> None:
    if a in container:
        _fail(reason, f"{a!r} in container")


def is_none(a: Any, reason: Optional[str] = None) -> None:
    if a is not None:
        _fail(reason, f"{a!r} is not None")


def is_not_none(a: Any, reason: Optional[str] = None) -> None:
    if a is None:
        _fail(reason, "value is None")


def is_instance(a: Any, typ: Any, reason: Optional[str] = None) -> None:
    if not isinstance(a, typ):
        _fail(reason, f"{type(a).__name__} is not an instance of {typ}")


def len_eq(a: Any, n: int, reason: Optional[str] = None) -> None:
    if len(a) != n:
        _fail(reason, f"len {len(a)} != {n}")
