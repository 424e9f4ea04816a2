"""Runs the S1 scatter microbenchmark (tools/s1mb.hip) on synthetic text."""
import ctypes
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "tests"))
import datagen  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 400_000_000
t = datagen.text(n)
L = ctypes.CDLL(os.path.join(os.path.dirname(__file__), "libs1mb.so"))
L.s1mb(ctypes.c_char_p(t), ctypes.c_uint32(n))
