"""A/B of libhbx builds on one box, alternating (GPU box): each round runs the same tools/ script once per
library, in a child process (HBX_LIB_PATH; "tree" = the in-tree build), and prints the script's last line:
    python tools/lib_ab.py ROUNDS LIB[,LIB...] SCRIPT [ARGS...]      (LIB: tree | ab/libhbx_<name>.so)"""
import os
import subprocess
import sys


def main():
    rounds = int(sys.argv[1])
    libs = sys.argv[2].split(",")
    cmd = [sys.executable, "-u"] + sys.argv[3:]
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    for r in range(rounds):
        for lib in libs:
            env = dict(os.environ)
            env.pop("HBX_LIB_PATH", None)
            if lib != "tree":
                env["HBX_LIB_PATH"] = os.path.join(root, lib)
            p = subprocess.run(cmd, cwd=root, env=env, capture_output=True, text=True, timeout=600)
            last = (p.stdout.strip().splitlines() or [""])[-1]
            print("round %d lib %s rc %d: %s" % (r, lib, p.returncode, last), flush=True)
            if p.returncode != 0:
                print(p.stderr[-2000:], flush=True)
                sys.exit(p.returncode)


if __name__ == "__main__":
    main()
