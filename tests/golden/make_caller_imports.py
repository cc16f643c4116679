"""Fixture generator: every ``src`` import of the reference's caller scripts.

Run here (where /root/reference exists):  python tests/golden/make_caller_imports.py
Writes tests/golden/caller_imports.json: for each top-level script of the reference
that imports from its ``src`` package (extract_features*.py, demo_isl_translate*.py,
the demos, ISL_extract_features_videos.py ...), the (line, module, names) of each
``from src.X import Y`` / ``from src import Y`` / ``import src.X``.  The scripts are
parsed with ``ast``, never executed.  Also lists which ``src`` modules the reference
ships, so tests/test_caller_seam.py can tell a replaced module from a fall-through one.
"""
import ast
import glob
import json
import os

REF = "/root/reference"
OUT = os.path.join(os.path.dirname(os.path.abspath(__file__)), "caller_imports.json")


def scan(path):
    tree = ast.parse(open(path, encoding="utf-8", errors="replace").read())
    out = []
    for node in ast.walk(tree):
        if isinstance(node, ast.ImportFrom) and node.module and (node.module == "src" or node.module.startswith("src.")):
            out.append({"line": node.lineno, "module": node.module, "names": [a.name for a in node.names]})
        elif isinstance(node, ast.Import):
            for a in node.names:
                if a.name == "src" or a.name.startswith("src."):
                    out.append({"line": node.lineno, "module": a.name, "names": []})
    return sorted(out, key=lambda e: e["line"])


def main():
    scripts = {}
    for p in sorted(glob.glob(os.path.join(REF, "*.py"))) + [os.path.join(REF, "src", "dataloader.py")]:
        imps = scan(p)
        if imps:
            scripts[os.path.relpath(p, REF)] = imps
    modules = sorted(os.path.splitext(os.path.basename(f))[0] for f in glob.glob(os.path.join(REF, "src", "*.py")))
    json.dump({"source": "ast scan of /root/reference scripts (tests/golden/make_caller_imports.py)",
               "reference_src_modules": modules, "scripts": scripts}, open(OUT, "w"), indent=1)
    print("wrote", OUT, len(scripts), "scripts")


if __name__ == "__main__":
    main()
