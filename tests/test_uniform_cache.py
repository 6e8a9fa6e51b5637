"""The Python mirror's uniform / texture value cache (babylon_pt.Effect, StreamPlayer.play_call): a
set that repeats the last value's float32 bits is skipped, anything else reaches the C ABI. Runs on
the CPU against a recording stand-in for libpt's setters (no device call)."""
import ctypes
import struct

import pytest

import babylon_pt as bp


class _Lib:
    def __init__(self):
        self.calls = []

    def pt_set_float(self, fx, name, arr, n):
        self.calls.append(("f", name.decode(), bytes(ctypes.cast(arr, ctypes.POINTER(ctypes.c_float * n)).contents)))
        return 0

    def pt_set_int(self, fx, name, v):
        self.calls.append(("i", name.decode(), v))
        return 0

    def pt_set_texture(self, fx, name, h):
        self.calls.append(("t", name.decode(), h))
        return 0


class _Engine:
    def check(self, rc, what=""):
        assert rc == 0, what
        return rc


class _Tex:
    def __init__(self, h):
        self.handle = h


@pytest.fixture
def fx(monkeypatch):
    fake = _Lib()
    monkeypatch.setattr(bp, "lib", lambda: fake)
    e = bp.Effect(_Engine(), 1)
    e.fake = fake
    return e


def _f32(*v):
    return struct.pack("%df" % len(v), *v)


def test_repeated_float_sets_are_skipped(fx):
    fx.setFloat("uA", 0.5)
    fx.setFloat("uA", 0.5)
    fx.setFloat2("uB", 1.0, 2.0)
    fx.setFloat2("uB", 1.0, 2.0)
    fx.setFloat("uA", 0.25)
    assert fx.fake.calls == [("f", "uA", _f32(0.5)), ("f", "uB", _f32(1.0, 2.0)), ("f", "uA", _f32(0.25))]


def test_cache_compares_float32_bits(fx):
    """-0.0 after 0.0 is a new value (== would call them equal), a NaN repeated with the same bits is
    the same value (== would call it new), and two doubles that round to the same float32 are one
    value."""
    fx.setFloat("u", 0.0)
    fx.setFloat("u", -0.0)
    fx.setFloat("u", float("nan"))
    fx.setFloat("u", float("nan"))
    fx.setFloat("u", 0.1)
    fx.setFloat("u", 0.1 + 1e-12)
    kinds = [c[2] for c in fx.fake.calls]
    assert kinds == [_f32(0.0), _f32(-0.0), _f32(float("nan")), _f32(0.1)]


def test_ints_and_textures(fx):
    fx.setInt("uI", 3)
    fx.setInt("uI", 3)
    fx.setBool("uI", True)
    a, b = _Tex(11), _Tex(12)
    fx.setTexture("s", a)
    fx.setTexture("s", a)
    fx.setTexture("s", b)
    a.handle = None           # disposed: the same object now binds nothing
    fx.setTexture("s", a)
    fx.setTexture("s", a)
    fx.setTexture("s", None)
    fx.setTexture("s", None)
    assert fx.fake.calls == [("i", "uI", 3), ("i", "uI", 1), ("t", "s", 11), ("t", "s", 12), ("t", "s", None),
                             ("t", "s", None)]


def test_recorded_entries_and_direct_setters(fx):
    """A recorded entry set again as the same object is skipped without packing; a direct setter in
    between (another value for that uniform) makes the next replay of the entry set it again."""
    ent = ["f", [2.0]]
    fx._set_entry("u", ent)
    fx._set_entry("u", ent)
    fx.setFloat("u", 3.0)
    fx._set_entry("u", ent)
    fx._set_entry("u", ["f", [2.0]])   # another object, same bits: the bit cache skips it
    ient = ["i", [7]]
    fx._set_entry("k", ient)
    fx._set_entry("k", ient)
    assert fx.fake.calls == [("f", "u", _f32(2.0)), ("f", "u", _f32(3.0)), ("f", "u", _f32(2.0)), ("i", "k", 7)]
