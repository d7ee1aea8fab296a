#!/usr/bin/env python3
"""Copy the reference's splitmix64 (struct splitmix64 { ... };,
/root/reference/unittest.cpp:24-35) verbatim into a build directory OUTSIDE
the repository, for oracle/ref/fpkey_shim.cpp to compile.  The reference's
unittest.cpp as a whole needs Orochi, <Windows.h> and <ppl.h> (absent), so
only this self-contained struct is taken.  Test infrastructure only.

usage: extract_splitmix64.py <unittest.cpp> <out.inc>"""
import sys

src, dst = sys.argv[1], sys.argv[2]
lines = open(src, encoding="utf-8", errors="replace").read().splitlines()
start = next(i for i, l in enumerate(lines) if l.strip().startswith("struct splitmix64"))
end = next(i for i in range(start, len(lines)) if lines[i].strip() == "};")
with open(dst, "w") as f:
    f.write(f"// extracted from {src}:{start + 1}-{end + 1} by oracle/ref/extract_splitmix64.py\n")
    f.write("\n".join(lines[start:end + 1]) + "\n")
print(f"splitmix64: {src}:{start + 1}-{end + 1} -> {dst}")
