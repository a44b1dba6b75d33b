"""dev.zarr.zarrjava.ZarrException (M/ZarrException.java:3-11) and the C-ABI status map."""


class ZarrException(Exception):
    """Data / format errors; message text follows the reference where one exists."""


class UnsupportedChainError(ZarrException):
    """The codec chain is valid but not device-supported (ZH_EUNSUPPORTED): the Java
    integration keeps the reference codec for it."""


def raise_for(err):
    """Map a _lib.ZhError to the reference's exception types."""
    from . import _abi as A
    st = getattr(err, "status", None)
    msg = str(err)
    if st == A.ZH_EDATA:
        e = ZarrException(msg)
        # where the failing chunk sits in a sequential read (zh_last_data_error): the
        # multi-rank read orders the ranks' errors by it (zarrhip.parallel.pick_error)
        e.position = getattr(err, "position", None)
        raise e from None
    if st == A.ZH_EUNSUPPORTED:
        raise UnsupportedChainError(msg) from None
    if st == A.ZH_EINVAL:
        raise ValueError(msg) from None
    if st == A.ZH_EARITH:
        raise ArithmeticError(msg) from None
    if st == A.ZH_EIO:  # a store file could not be read (StoreException.readFailed)
        from .store import StoreException
        raise StoreException(msg) from None
    raise RuntimeError(msg) from None
