"""Tiny exact-match file patcher used during development: fails loudly when a pattern is absent."""
import sys


def patch(path, pairs):
    s = open(path).read()
    for a, b in pairs:
        if a not in s:
            raise SystemExit(f"pattern not found in {path}: {a[:80]!r}")
        s = s.replace(a, b)
    open(path, "w").write(s)


if __name__ == "__main__":
    # usage: edit.py FILE OLD NEW [OLD NEW ...]
    args = sys.argv[2:]
    assert len(args) % 2 == 0, "pairs of OLD NEW expected"
    patch(sys.argv[1], list(zip(args[0::2], args[1::2])))
