"""Every path a committed profile summary cites as its source exists, so
pruning or bundling raw passes can never leave a summary pointing at nothing (CPU only).

Sources are the strings under keys named like "*source*" in every JSON file under profiles/
(summaries, bench records). A path is either a file or directory in the tree, or
"<bundle>.bundle.json#<prefix>" -- a raw pass directory packed by tools/bundle_profiles.py, which
must hold at least one file under <prefix>. Scratch paths a run printed (gpurun_out/...) must map
to the committed copy named in ALIASES."""
import json
import pathlib
import re

import pytest

ROOT = pathlib.Path(__file__).resolve().parent.parent
PROFILES = ROOT / "profiles"
TOKEN = re.compile(r"(?:profiles|gpurun_out|tools|tests)/[\w./\-#<>,]+")
# round 1's v17 bench record names the scratch directory its PMC run wrote; the committed copy:
ALIASES = {"gpurun_out/ev_v17/pmc_uniform": "profiles/r01/v17_pmc_uniform"}


def _sources():
    out = []
    for f in sorted(PROFILES.rglob("*.json")):
        if f.name.endswith(".bundle.json"):
            continue
        try:
            d = json.loads(f.read_text())
        except ValueError:
            continue

        def walk(x, key=None):
            if isinstance(x, dict):
                for k, v in x.items():
                    walk(v, k)
            elif isinstance(x, list):
                for v in x:
                    walk(v, key)
            elif isinstance(x, str) and key and "source" in key:
                out.extend((f.relative_to(ROOT).as_posix(), t.rstrip(".,")) for t in TOKEN.findall(x))
        walk(d)
    return out


SOURCES = _sources()
_bundles = {}


def _resolves(path):
    path = ALIASES.get(path.rstrip("/"), path)
    if "#" in path:
        b, prefix = path.split("#", 1)
        if b not in _bundles:
            f = ROOT / b
            _bundles[b] = json.loads(f.read_text())["files"] if f.exists() else None
        return _bundles[b] is not None and any(k.startswith(prefix) for k in _bundles[b])
    if (ROOT / path).exists():
        return True
    # a record written before its source directory was bundled cites the directory's old path
    parts = path.rstrip("/").split("/")
    for i in range(len(parts) - 1, 1, -1):
        b = "/".join(parts[:i]) + ".bundle.json"
        if (ROOT / b).exists():
            return _resolves(b + "#" + "/".join(parts[i:]))
    return False


def test_summaries_cite_sources():
    assert len(SOURCES) > 500  # the 27 PMC summaries alone cite 7 passes each
    assert any("#" in s for _, s in SOURCES)


def test_every_cited_source_exists():
    missing = [(f, s) for f, s in SOURCES if not _resolves(s)]
    assert not missing, missing[:20]


def test_headline_summary_sources_are_its_seven_passes():
    prof = json.loads((PROFILES / "pmc_uniform.json").read_text())
    srcs = prof["source"].split()
    assert len(srcs) == 7 and all(_resolves(s) for s in srcs)


@pytest.mark.parametrize("bundle", sorted(p.relative_to(ROOT).as_posix() for p in PROFILES.rglob("*.bundle.json")))
def test_bundles_hold_text_files(bundle):
    b = json.loads((ROOT / bundle).read_text())
    assert b["bundled_from"] + ".bundle.json" == bundle and b["files"]
