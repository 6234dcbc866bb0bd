"""Build the product library of an earlier commit as a tuning variant (same-box A/B against history):
the commit's hslabs_amd/csrc and include/ are extracted with `git archive` into tools/_build/prev_<name>/
and compiled by hslabs_amd/build.py's own recipe into hslabs_amd/_build/variants/libhslabs_<name>.so
(select it with HSLABS_VARIANT=<name>). The commit must export the current ABI (hs_run_args layout).

  python tools/build_prev.py <commit> <name>
"""
import os
import shutil
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    commit, name = sys.argv[1], sys.argv[2]
    dst = os.path.join(ROOT, "tools", "_build", f"prev_{name}")
    shutil.rmtree(dst, ignore_errors=True)
    os.makedirs(dst)
    tar = subprocess.run(["git", "-C", ROOT, "archive", commit, "hslabs_amd/csrc", "include"], check=True,
                         capture_output=True).stdout
    subprocess.run(["tar", "-x", "-C", dst], input=tar, check=True)
    from hslabs_amd import build as B
    B.SRC = os.path.join(dst, "hslabs_amd", "csrc")
    out = B._compile(os.path.join(B.VARIANT_DIR, f"libhslabs_{name}.so"))
    B._isa_check(out, fatal=False)
    print(out)


if __name__ == "__main__":
    main()
