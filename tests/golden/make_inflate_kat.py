"""Generate tests/golden/inflate_kat.json from the reference's decoder known-answer tests.

Run here (in the build container, where /root/reference exists):
    python tests/golden/make_inflate_kat.py
The output is DATA only: for each deterministic @Test in
/root/reference/test/io/nayuki/deflate/InflaterInputStreamTest.java it records the test name,
its source line, the input bit string (stream order, spaces stripped) and either the expected
output hex or the expected DataFormatException.Reason.  The three randomized generators
(:131, :166, :306) are restated with a seeded RNG in tests/test_oracle_inflate.py instead.
"""
import json
import os
import re
import sys

REF = "/root/reference/test/io/nayuki/deflate/InflaterInputStreamTest.java"
OUT = os.path.join(os.path.dirname(os.path.abspath(__file__)), "inflate_kat.json")


def parse_expr(expr, env):
    """Evaluate a Java string expression made of literals, variables and '+'."""
    parts = []
    for tok in re.findall(r'"((?:[^"\\]|\\.)*)"|([A-Za-z_]\w*)', expr):
        lit, var = tok
        if var:
            parts.append(env[var])
        else:
            parts.append(lit)
    return "".join(parts)


def main():
    src = open(REF).read()
    lines = src.split("\n")
    out = []
    # Split into methods at "@Test"
    starts = [i for i, l in enumerate(lines) if "@Test" in l]
    for si, start in enumerate(starts):
        end = starts[si + 1] if si + 1 < len(starts) else len(lines)
        body = "\n".join(lines[start:end])
        m = re.search(r"public void (test\w+)\(\)", body)
        name = m.group(1)
        if "rand." in body.split("private static void test(")[0] and "TRIALS" in body:
            continue  # randomized generator: restated separately
        env = {}
        for vm in re.finditer(r'String (\w+) = ((?:"(?:[^"\\]|\\.)*"\s*\+?\s*)+);', body):
            env[vm.group(1)] = parse_expr(vm.group(2), env)
        cm = re.search(r"\b(test|testFail)\((.*?),\s*(Reason\.\w+|\"[^\"]*\")\);", body, re.S)
        kind, arg1, arg2 = cm.group(1), cm.group(2), cm.group(3)
        bits = parse_expr(arg1, env).replace(" ", "")
        assert re.fullmatch(r"[01]*", bits), (name, bits)
        rec = {"name": name, "line": start + 1, "bits": bits}
        if kind == "test":
            rec["expect_hex"] = arg2.strip('"').replace(" ", "").lower()
            rec["expect_reason"] = None
        else:
            rec["expect_hex"] = None
            rec["expect_reason"] = arg2.split(".")[1]
        out.append(rec)
    with open(OUT, "w") as f:
        json.dump({"source": "T/InflaterInputStreamTest.java", "tests": out}, f, indent=1)
    print(f"wrote {len(out)} known-answer tests to {OUT}", file=sys.stderr)


if __name__ == "__main__":
    main()
