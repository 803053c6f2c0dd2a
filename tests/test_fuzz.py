"""The wire codecs (gojson.hpp, lsp_message.cpp, bitcoin.cpp) under a
coverage-guided fuzzer and against an independent JSON grammar.

- `make fuzz` builds tests/fuzz/fuzz_codecs.cpp with libFuzzer + ASan +
  UBSan; here it runs for 6 s from the seeds in tests/fuzz/seeds (a longer
  run: tools/fuzz.sh).  Properties: no sanitizer report; a syntax error
  leaves the message untouched; any other input re-encodes to an error-free
  fixed point; base64 decode(encode(decode(s))) == decode(s).
- Go's scanner grammar (stage 1 of Unmarshal) against Python's json module
  on random JSON-like inputs: for valid UTF-8 without NaN/Infinity (which
  Python accepts and Go does not), `p1miner json` answers "ERROR" exactly
  when json.loads raises."""
import json
import os
import random
import shutil
import subprocess

import pytest

from conftest import ROOT

FUZZ = os.path.join(ROOT, "build", "san", "fuzz_codecs")
MINER = os.path.join(ROOT, "p1_amd", "p1miner")
SANCXX = "/opt/rocm/lib/llvm/bin/clang++"


@pytest.mark.skipif(not os.path.exists(SANCXX), reason="ROCm clang (libFuzzer runtime) not present")
def test_codec_fuzzer_6s(tmp_path):
    subprocess.run(["make", "-s", "-C", ROOT, "fuzz"], check=True, stdout=subprocess.DEVNULL)
    corpus = tmp_path / "corpus"
    shutil.copytree(os.path.join(ROOT, "tests", "fuzz", "seeds"), corpus)
    r = subprocess.run([FUZZ, "-max_total_time=6", "-print_final_stats=1", "-max_len=4096", str(corpus)],
                       capture_output=True, text=True, timeout=120, cwd=tmp_path)
    assert r.returncode == 0, r.stderr[-4000:]
    runs = [ln for ln in r.stderr.splitlines() if ln.startswith("stat::number_of_executed_units")]
    assert runs and int(runs[0].split()[-1]) > 10000, r.stderr[-2000:]


@pytest.mark.skipif(not os.path.exists(SANCXX), reason="ROCm clang (libFuzzer runtime) not present")
def test_planner_fuzzer_6s(tmp_path):
    """planner.hpp (make_plan, plan_shards) on fuzzer-chosen lengths, ranges
    near decade edges and the u64 top, shard counts and planner switches
    (tests/fuzz/fuzz_planner.cpp): every plan succeeds and hashes exactly
    upper-lower+1 nonces; shards are in order, contiguous and cover the range."""
    subprocess.run(["make", "-s", "-C", ROOT, "fuzz"], check=True, stdout=subprocess.DEVNULL)
    r = subprocess.run([os.path.join(ROOT, "build", "san", "fuzz_planner"), "-max_total_time=6", "-seed=440",
                        "-print_final_stats=1"], capture_output=True, text=True, timeout=120, cwd=tmp_path)
    assert r.returncode == 0, r.stderr[-4000:]
    runs = [ln for ln in r.stderr.splitlines() if ln.startswith("stat::number_of_executed_units")]
    assert runs and int(runs[0].split()[-1]) > 2000, r.stderr[-2000:]


ATOMS = ['{', '}', '[', ']', ',', ':', '"', '"a"', '"Type"', '"Data"', '"Lower"', '1', '0', '-', '01', '1.5', '1.',
         '1e5', '1E+2', '-0', 'true', 'false', 'null', 'nul', ' ', '\t', '\n', '\\', '\\u00e9', '\\ud800', '\\x',
         'é', ' ', '\x01', "'", '"\\"', '"\\\\"', '"\\/"', '"\\u12"', '2e', '.5']


def random_doc(rnd):
    if rnd.random() < 0.5:  # a valid document, possibly mutated
        def val(d):
            k = rnd.randrange(7 if d < 4 else 4)
            if k == 0:
                return str(rnd.choice([0, 1, -1, 12, 2**64, -2**63, 1.5, 1e300]))
            if k == 1:
                return json.dumps(rnd.choice(["", "x", "é", " ", "a\"b", "\\", "\x01", "😀"]),
                                  ensure_ascii=rnd.random() < 0.5)
            if k == 2:
                return rnd.choice(["true", "false", "null"])
            if k == 3:
                return '"%s"' % rnd.choice(["Type", "Data", "Lower"])
            if k in (4, 5):
                return "{" + ",".join('"%s":%s' % (rnd.choice(["Type", "Data", "Lower", "Upper", "x"]), val(d + 1))
                                      for _ in range(rnd.randrange(4))) + "}"
            return "[" + ",".join(val(d + 1) for _ in range(rnd.randrange(4))) + "]"
        s = val(0)
        for _ in range(rnd.randrange(3)):
            i = rnd.randrange(len(s) + 1)
            op = rnd.randrange(3)
            if op == 0:
                s = s[:i] + rnd.choice(ATOMS) + s[i:]
            elif op == 1 and s:
                s = s[:i] + s[i + 1:]
            else:
                s = s[:i] + rnd.choice(ATOMS) + s[i + 1:]
        return s
    return "".join(rnd.choice(ATOMS) for _ in range(rnd.randrange(1, 12)))


def test_syntax_check_matches_python_json():
    rnd = random.Random(440)
    docs = []
    while len(docs) < 4000:
        s = random_doc(rnd)
        if "\n" in s or "\r" in s or "NaN" in s or "Infinity" in s:
            continue  # one document per line; NaN/Infinity are Python extensions
        try:
            s.encode("utf-8")
        except UnicodeEncodeError:
            continue  # lone surrogates from the generator
        docs.append(s)
    r = subprocess.run([MINER, "json"], input="\n".join(docs) + "\n", capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stderr
    out = r.stdout.split("\n")
    n_valid = 0
    for s, o in zip(docs, out):
        try:
            json.loads(s)
            ok = True
        except ValueError:
            ok = False
        n_valid += ok
        assert (o != "ERROR") == ok, (s, o)
    assert 500 < n_valid < len(docs) - 500  # both outcomes well represented
