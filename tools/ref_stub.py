"""Container-only loader for the reference scripts (TEST TOOLING, never shipped).

The reference (`/root/reference/pypanadapter_spectrum.py`, `pypanadapter_thread.py`)
imports PyQt5 / pyqtgraph at module level (S:15, S:27).  Neither is installed, so
this module registers permissive stand-in modules in `sys.modules` and then loads
the reference files *unmodified* with importlib.  Only
`tools/gen_golden.py` uses it, and only when `/root/reference` exists.
"""
from __future__ import annotations

import importlib.util
import os
import sys
import types

REF_DIR = "/root/reference"


class _Meta(type):
    def __getattr__(cls, name):  # lets `class X(QtWidgets.QDialog)` and X.attr work
        return _Any


class _Any(metaclass=_Meta):
    def __init__(self, *a, **k):
        pass

    def __call__(self, *a, **k):
        # decorator form (`@QtCore.pyqtSlot(...)`) hands the function back unchanged
        if len(a) == 1 and callable(a[0]) and not k:
            return a[0]
        return _Any()

    def __getattr__(self, name):
        return _Any()

    def __iter__(self):
        return iter(())

    def __bool__(self):
        return False


def _install_qt_stubs() -> None:
    names = ["PyQt5", "PyQt5.QtCore", "PyQt5.QtWidgets", "PyQt5.QtGui",
             "PyQt5.QtDBus", "pyqtgraph"]
    for n in names:
        if n in sys.modules:
            continue
        m = types.ModuleType(n)
        m.__getattr__ = lambda attr: _Any  # noqa: E731  (module-level getattr)
        sys.modules[n] = m
    pyqt = sys.modules["PyQt5"]
    for sub in ("QtCore", "QtWidgets", "QtGui", "QtDBus"):
        setattr(pyqt, sub, sys.modules["PyQt5." + sub])


def load(variant: str = "spectrum"):
    """Load `pypanadapter_<variant>.py` from the read-only reference tree."""
    if not os.path.isdir(REF_DIR):
        raise FileNotFoundError(REF_DIR)
    _install_qt_stubs()
    sys.dont_write_bytecode = True
    if REF_DIR not in sys.path:  # T imports `newtrap` from the same directory
        sys.path.append(REF_DIR)
    name = f"pypanadapter_{variant}"
    if name in sys.modules:
        return sys.modules[name]
    spec = importlib.util.spec_from_file_location(name, os.path.join(REF_DIR, name + ".py"))
    mod = importlib.util.module_from_spec(spec)
    sys.modules[name] = mod
    spec.loader.exec_module(mod)
    return mod


class Capture:
    """Stand-in for Qt widgets the reference's update() touches; records calls."""

    def __init__(self):
        self.calls = []

    def image_update(self, psd):
        self.calls.append(("image_update", psd.copy()))

    def setData(self, *a, **k):
        self.calls.append(("setData",) + tuple(x.copy() if hasattr(x, "copy") else x for x in a))

    def setWindowTitle(self, title):
        self.calls.append(("title", title))
