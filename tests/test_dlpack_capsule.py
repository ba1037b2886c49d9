"""The DLPack capsule destructor of _capi.Handle.output_dlpack (CPU, no device):
a capsule dropped unconsumed calls the managed tensor's deleter; one a consumer
has taken (renamed "used_dltensor") does not."""
import ctypes
import gc

import pkgload


def _capsule(name, calls):
    from marl_traffic_intersection_amd import _capi

    @_capi._DL_DELETER
    def deleter(ptr):
        calls.append(ptr)

    m = _capi._DLManaged()
    m.deleter = ctypes.cast(deleter, ctypes.c_void_p)
    new = ctypes.pythonapi.PyCapsule_New
    new.restype = ctypes.py_object
    new.argtypes = [ctypes.c_void_p, ctypes.c_char_p, ctypes.c_void_p]
    cap = new(ctypes.addressof(m), _capi._DLTENSOR, ctypes.cast(_capi._capsule_destructor, ctypes.c_void_p))
    if name != _capi._DLTENSOR:
        ctypes.pythonapi.PyCapsule_SetName.argtypes = [ctypes.py_object, ctypes.c_char_p]
        ctypes.pythonapi.PyCapsule_SetName(cap, name)
    return cap, m, deleter


def test_unconsumed_capsule_calls_deleter():
    pkgload.load()
    calls = []
    cap, m, keep = _capsule(b"dltensor", calls)
    addr = ctypes.addressof(m)
    del cap
    gc.collect()
    assert calls == [addr]


def test_consumed_capsule_leaves_deleter_to_consumer():
    pkgload.load()
    calls = []
    cap, m, keep = _capsule(b"used_dltensor", calls)
    del cap
    gc.collect()
    assert calls == []
