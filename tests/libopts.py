"""The library's tuning switches in tests (include/contivcls.h
cls_engine_set_option; cls_compile_v4 / v16 take them as an option string).

The library never reads the process environment.  A test sets a switch with
the ``libopt`` fixture (conftest.py): ``libopt.set(key, value, *engines)``
applies it to the engines given and to every ``cls_image.compile_blob`` call
of the test; the fixture restores the defaults afterwards.
"""

CURRENT = {}     # key -> value for compile_blob's option string


def option_string(extra=None) -> bytes:
    d = dict(CURRENT)
    d.update(extra or {})
    return ",".join("%s=%s" % kv for kv in d.items()).encode()


class LibOpts:
    def __init__(self):
        self._set = []           # (engine, key) to restore

    def set(self, key, value, *engines):
        CURRENT[key] = str(value)
        for e in engines:
            e.set_option(key, value)
            self._set.append((e, key))

    def undo(self):
        for e, k in reversed(self._set):
            if getattr(e, "h", None):
                e.set_option(k, None)
        self._set.clear()
        CURRENT.clear()
