"""Training lengths in records / batches / epochs (reference ``master/pkg/model/length.go``)."""
from typing import Any, Dict, Union

RECORDS = "records"
BATCHES = "batches"
EPOCHS = "epochs"
UNITS = (RECORDS, BATCHES, EPOCHS)


class UnitContext:
    def __init__(self, default_unit: str, global_batch_size: int, records_per_epoch: int) -> None:
        self.default_unit = default_unit
        self.global_batch_size = int(global_batch_size)
        self.records_per_epoch = int(records_per_epoch)


class Length:
    __slots__ = ("unit", "units")

    def __init__(self, unit: str, units: int) -> None:
        if unit not in UNITS:
            raise ValueError(f"invalid length unit {unit!r}")
        self.unit = unit
        self.units = int(units)

    @staticmethod
    def parse(v: Union[Dict[str, Any], "Length"]) -> "Length":
        if isinstance(v, Length):
            return v
        if not isinstance(v, dict):
            raise ValueError(f"invalid length: {v!r}")
        keys = [k for k in UNITS if k in v]
        if len(keys) != 1 or len(v) != 1:
            raise ValueError(f"invalid length: {v!r}")
        return Length(keys[0], int(v[keys[0]]))

    def to_json(self) -> Dict[str, int]:
        return {self.unit: self.units}

    def __json__(self) -> Dict[str, int]:
        return self.to_json()

    def __eq__(self, o: object) -> bool:
        return isinstance(o, Length) and o.unit == self.unit and o.units == self.units

    def __hash__(self) -> int:
        return hash((self.unit, self.units))

    def __repr__(self) -> str:
        return f"{self.units} {self.unit}"

    def _same(self, o: "Length") -> None:
        if o.unit != self.unit:
            raise ValueError(f"unit mismatch {self.unit} vs {o.unit}")

    def __add__(self, o: "Length") -> "Length":
        self._same(o)
        return Length(self.unit, self.units + o.units)

    def __sub__(self, o: "Length") -> "Length":
        self._same(o)
        return Length(self.unit, self.units - o.units)

    def mult_int(self, k: int) -> "Length":
        return Length(self.unit, self.units * k)

    def div_int(self, k: int) -> "Length":
        return Length(self.unit, self.units // k)

    def to_nearest_batch(self, ctx: UnitContext) -> int:
        if self.unit == RECORDS:
            return self.units // ctx.global_batch_size
        if self.unit == BATCHES:
            return self.units
        return (self.units * ctx.records_per_epoch) // ctx.global_batch_size

    def equal_within_batch(self, batches: int, ctx: UnitContext) -> bool:
        if self.unit == RECORDS:
            return abs(self.units - batches * ctx.global_batch_size) < ctx.global_batch_size
        if self.unit == BATCHES:
            return self.units == batches
        return abs(self.units * ctx.records_per_epoch - batches * ctx.global_batch_size) < ctx.global_batch_size


def units_from_batches(batches: int, ctx: UnitContext) -> float:
    if ctx.default_unit == RECORDS:
        return float(batches * ctx.global_batch_size)
    if ctx.default_unit == BATCHES:
        return float(batches)
    return float(batches * ctx.global_batch_size) / float(ctx.records_per_epoch)
