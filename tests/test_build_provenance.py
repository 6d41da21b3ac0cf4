"""Build provenance: the in-tree extension carries the content hash of the
csrc/ sources it was linked from, the build is a no-op exactly when that hash matches, and
ops.hip refuses to load a binary built from other sources. No GPU needed: importing the
extension does not touch the device."""

import importlib
import os

import pytest

from distributed_learning_simulator_amd.ops import build


def test_source_hash_tracks_content(tmp_path, monkeypatch):
    h0 = build.source_hash()
    assert h0 == build.source_hash() and len(h0) == 20
    # a copy of csrc/ with one byte changed hashes differently
    src = tmp_path / "csrc"
    src.mkdir()
    for f in os.listdir(build.CSRC):
        (src / f).write_bytes(open(os.path.join(build.CSRC, f), "rb").read())
    monkeypatch.setattr(build, "CSRC", str(src))
    assert build.source_hash() == h0
    p = src / "common.h"
    p.write_bytes(p.read_bytes() + b"\n")
    assert build.source_hash() != h0


def test_built_binary_matches_tree():
    build.build()
    assert build.is_current()
    torch = pytest.importorskip("torch")  # noqa: F841  (the HIP runtime is loaded through torch)
    C = importlib.import_module("distributed_learning_simulator_amd._dls_hip")
    assert C.src_hash() == build.source_hash()


def test_stale_binary_is_refused(monkeypatch):
    pytest.importorskip("torch")
    from distributed_learning_simulator_amd.ops import hip

    monkeypatch.setattr(build, "source_hash", lambda: "0" * 20)
    with pytest.raises(ImportError, match="different sources"):
        hip._check_provenance()
