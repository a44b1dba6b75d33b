"""v3 DataType (M/v3/DataType.java:5-68): name, byte count, numpy dtype of the decoded
elements (host little-endian, as ucar.ma2 holds them)."""
import enum

import numpy as np


class DataType(enum.Enum):
    BOOL = ("bool", 1, np.bool_)
    INT8 = ("int8", 1, np.int8)
    INT16 = ("int16", 2, np.dtype("<i2"))
    INT32 = ("int32", 4, np.dtype("<i4"))
    INT64 = ("int64", 8, np.dtype("<i8"))
    UINT8 = ("uint8", 1, np.uint8)
    UINT16 = ("uint16", 2, np.dtype("<u2"))
    UINT32 = ("uint32", 4, np.dtype("<u4"))
    UINT64 = ("uint64", 8, np.dtype("<u8"))
    FLOAT32 = ("float32", 4, np.dtype("<f4"))
    FLOAT64 = ("float64", 8, np.dtype("<f8"))

    @property
    def value_name(self):
        return self.value[0]

    def getByteCount(self):
        return self.value[1]

    @property
    def numpy(self):
        return np.dtype(self.value[2])

    @classmethod
    def of(cls, name):
        for d in cls:
            if d.value[0] == name:
                return d
        raise ValueError(f"Unknown data type '{name}'")
