#!/usr/bin/env python3
"""Pack raw rocprofv3 pass directories under profiles/ into one JSON bundle each (VERDICT r5
next #6: the evidence stays, the file count does not grow by hundreds per round).

For every directory D given, writes D.bundle.json = {"bundled_from": D, "files": {relative path:
text}} with every file under D (pass lines, side files, kernel traces, the measured dispatch's
counter rows), removes D, and rewrites every reference "D/<rest>" in the tracked text files under
profiles/ (and DESIGN.md) to "D.bundle.json#<rest>". tests/test_profile_sources.py resolves both
forms. tools/bundle_profiles.py --extract B.bundle.json DEST unpacks a bundle again.
Usage: python3 tools/bundle_profiles.py DIR [DIR ...]
"""
import json
import pathlib
import shutil
import sys

ROOT = pathlib.Path(__file__).resolve().parent.parent


def bundle(d):
    d = d.resolve()
    rel = d.relative_to(ROOT).as_posix()
    files = {p.relative_to(d).as_posix(): p.read_text() for p in sorted(d.rglob("*")) if p.is_file()}
    out = d.parent / (d.name + ".bundle.json")
    out.write_text(json.dumps({"bundled_from": rel, "files": files}, indent=0) + "\n")
    shutil.rmtree(d)
    return rel, out.relative_to(ROOT).as_posix(), len(files)


def rewrite(pairs):
    targets = [p for p in (ROOT / "profiles").rglob("*") if p.is_file() and p.suffix in (".json", ".md", ".txt")
               and not p.name.endswith(".bundle.json")] + [ROOT / "DESIGN.md"]
    for p in targets:
        s = p.read_text()
        t = s
        for rel, b in pairs:
            t = t.replace(rel + "/", b + "#")
        if t != s:
            p.write_text(t)


def extract(bundle_path, dest):
    b = json.loads(pathlib.Path(bundle_path).read_text())
    for name, text in b["files"].items():
        f = pathlib.Path(dest) / name
        f.parent.mkdir(parents=True, exist_ok=True)
        f.write_text(text)


if __name__ == "__main__":
    if sys.argv[1:2] == ["--extract"]:
        extract(sys.argv[2], sys.argv[3])
        sys.exit(0)
    pairs = []
    for a in sys.argv[1:]:
        rel, b, n = bundle(pathlib.Path(a))
        pairs.append((rel, b))
        print(f"{rel}: {n} files -> {b}")
    rewrite(pairs)
