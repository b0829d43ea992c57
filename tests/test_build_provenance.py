"""Build provenance: the loaded libgelim.so carries the digest of the sources
it was compiled from (csrc/cmake/source_digest.cmake); it must equal the
digest of csrc/ in this tree, so a stale or foreign prebuilt library cannot
pass the suite unnoticed."""
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))


def test_library_built_from_this_tree():
    from gelim import _native

    built, here = _native.build_digest(), _native.source_digest()
    assert len(built) == 64 and built == here, (
        f"libgelim.so was built from other sources (library {built[:12]}, tree {here[:12]}): "
        "rebuild with `python __graft_entry__.py build`")


def test_digest_tracks_source_edits(tmp_path):
    import shutil

    from gelim import _native

    csrc = tmp_path / "csrc"
    shutil.copytree(ROOT / "csrc", csrc)
    before = _native.source_digest(csrc)
    f = csrc / "hip" / "dgemm.hip"
    f.write_text(f.read_text() + "\n")
    assert _native.source_digest(csrc) != before
