"""build.py's flags stamp (CPU): written only after every object compiled and the library linked, and
removed when a compile fails — so an interrupted build after a flag change cannot leave objects of the old
flags looking current (round-4 advice).  A stand-in compiler script replaces hipcc; nothing real is built."""
import os
import stat

import pytest

from irm_motion_planning_amd import build


def _fake_hipcc(tmp_path, fail_on=None):
    """A compiler stand-in: creates the -o target, or exits 1 when an argument contains `fail_on`."""
    script = tmp_path / "fake_hipcc.sh"
    cond = f'case "$*" in *{fail_on}*) exit 1;; esac' if fail_on else ""
    script.write_text(f"""#!/bin/bash
{cond}
out=""
while [ $# -gt 0 ]; do
  if [ "$1" = "-o" ]; then out="$2"; shift; fi
  shift
done
touch "$out"
""")
    script.chmod(script.stat().st_mode | stat.S_IEXEC)
    return str(script)


def _variant(tmp_path, flags):
    # an absolute library path: build() joins it onto the package directory, which leaves it as it is
    build.VARIANTS["stamptest"] = (str(tmp_path / "libstamptest.so"), list(flags))


@pytest.fixture
def sandbox(tmp_path, monkeypatch):
    monkeypatch.setattr(build, "OBJ", str(tmp_path / "obj"))
    monkeypatch.setitem(build.VARIANTS, "stamptest", (str(tmp_path / "libstamptest.so"), ["-DIRM_STAMP_TEST"]))
    return tmp_path


def test_stamp_written_after_link(sandbox, monkeypatch):
    monkeypatch.setattr(build, "HIPCC", _fake_hipcc(sandbox))
    out = build.build(variant="stamptest", jobs=4)
    stamp = os.path.join(build.OBJ, "stamptest", "flags.txt")
    assert os.path.exists(out)
    assert open(stamp).read() == "\n".join(build.CFLAGS + ["-DIRM_STAMP_TEST"])


def test_failed_compile_leaves_no_stamp(sandbox, monkeypatch):
    monkeypatch.setattr(build, "HIPCC", _fake_hipcc(sandbox))
    build.build(variant="stamptest", jobs=4)
    stamp = os.path.join(build.OBJ, "stamptest", "flags.txt")
    assert os.path.exists(stamp)
    # a flag change followed by a failing compile: the stamp must not survive
    _variant(sandbox, ["-DIRM_STAMP_TEST", "-DIRM_STAMP_TEST2"])
    monkeypatch.setattr(build, "HIPCC", _fake_hipcc(sandbox, fail_on="opt_fix3_128"))
    with pytest.raises(Exception):
        build.build(variant="stamptest", jobs=4)
    assert not os.path.exists(stamp)
    # the next build with a working compiler rebuilds everything and stamps the new flags
    monkeypatch.setattr(build, "HIPCC", _fake_hipcc(sandbox))
    build.build(variant="stamptest", jobs=4)
    assert open(stamp).read() == "\n".join(build.CFLAGS + ["-DIRM_STAMP_TEST", "-DIRM_STAMP_TEST2"])
