"""ENVIRONMENT.md lists every ``HDS_*`` variable the package (and bench.py) reads: a knob added without a row fails
here."""
import os
import re

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
_READ = re.compile(r"""(?:environ\.get\(|getenv\(|environ\[)\s*["'](HDS_[A-Z0-9_]+)""")


def _read_vars():
    found = set()
    files = [os.path.join(ROOT, "bench.py")]
    for d, _, names in os.walk(os.path.join(ROOT, "hcache_deepspeed_amd")):
        files += [os.path.join(d, n) for n in names if n.endswith((".py", ".cpp", ".hip", ".h"))]
    for f in files:
        with open(f, encoding="utf-8", errors="replace") as fh:
            found.update(_READ.findall(fh.read()))
    return found


def test_every_env_knob_is_documented():
    with open(os.path.join(ROOT, "ENVIRONMENT.md"), encoding="utf-8") as fh:
        doc = set(re.findall(r"`(HDS_[A-Z0-9_]+)`", fh.read()))
    read = _read_vars()
    assert len(read) > 30  # the scan itself works
    assert not read - doc, sorted(read - doc)
