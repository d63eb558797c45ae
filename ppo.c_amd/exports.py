#!/usr/bin/env python3
"""List every function declared in include/*.h (the libppo C ABI).

Used by the Makefile to write the linker version script (only these symbols
are exported from libppo.so) and by tests/test_abi.py to check that the built
library exports each of them.
"""
import os
import re
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
INCLUDE = os.path.join(HERE, "..", "include")

_DECL = re.compile(r"^\s*(?:[A-Za-z_][\w\s\*]*?[\s\*])([A-Za-z_]\w*)\s*\([^;{]*\)\s*;", re.M)
_SKIP = {"if", "while", "for", "switch", "return", "sizeof"}


def _strip_comments(text):
    text = re.sub(r"/\*.*?\*/", " ", text, flags=re.S)
    return re.sub(r"//[^\n]*", " ", text)


def declared_functions(include_dir=INCLUDE):
    names = []
    for fn in sorted(os.listdir(include_dir)):
        if not fn.endswith(".h"):
            continue
        text = _strip_comments(open(os.path.join(include_dir, fn)).read())
        # drop typedef'd function-pointer struct members: they contain "(*"
        for m in _DECL.finditer(text):
            decl = m.group(0)
            name = m.group(1)
            if "(*" in decl or name in _SKIP or decl.lstrip().startswith("typedef"):
                continue
            names.append((fn, name))
    return names


def main():
    if len(sys.argv) > 1 and sys.argv[1] == "--map":
        names = sorted({n for _, n in declared_functions()})
        print("{\n  global:")
        for n in names:
            print(f"    {n};")
        print("  local: *;\n};")
    else:
        for fn, n in declared_functions():
            print(f"{fn}\t{n}")


if __name__ == "__main__":
    main()
