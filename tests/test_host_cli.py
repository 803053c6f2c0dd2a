"""The C++ host mirror of the reference's bitcoin package / miner loop
(p1_amd/host, binary p1_amd/p1miner)."""
import json
import os
import subprocess

import pytest

from conftest import ROOT

MINER = os.path.join(ROOT, "p1_amd", "p1miner")
U64_MAX = (1 << 64) - 1


@pytest.fixture(scope="module", autouse=True)
def built():
    if not os.path.exists(MINER):
        subprocess.run(["make", "-s", "-C", ROOT, "p1_amd/p1miner"], check=True)


def run(args, stdin=None):
    # one visible GPU: without --device the miner opens every visible device
    env = dict(os.environ, HIP_VISIBLE_DEVICES=os.environ.get("HIP_VISIBLE_DEVICES", "0").split(",")[0])
    return subprocess.run([MINER] + args, input=stdin, capture_output=True, text=True, timeout=600, env=env)


def test_json_wire_format_matches_go():
    # Go encoding/json of bitcoin.Message (message.go:18-23): field order,
    # HTML-safe escaping (< > &), uint64 as exact integers.
    lines = [
        '{"Type":1,"Data":"bradfitz","Lower":0,"Upper":9999,"Hash":0,"Nonce":0}',
        '{"type":2,"hash":18446744073709551615,"nonce":5}',       # Go matches keys case-insensitively
        '{"Type":1,"Data":"a<b>&\\"c\\\\ \\u00e9\\u0001\\u2028","Lower":1,"Upper":2}',
        '{"Type":0,"Extra":[1,{"x":null}],"Data":null}',          # unknown keys / null ignored
        '{"Type":1,"Lower":-1}',                                  # negative uint64: a type error
        '{"Type":1,"Upper":18446744073709551616}',                # overflow: a type error
    ]
    out = run(["json"], "\n".join(lines) + "\n").stdout.split("\n")
    assert out[0] == lines[0] + "\t[Request bradfitz 0 9999]"
    assert out[1] == '{"Type":2,"Data":"","Lower":0,"Upper":0,"Hash":18446744073709551615,"Nonce":5}' \
                     "\t[Result 18446744073709551615 5]"
    assert out[2].split("\t")[0] == \
        '{"Type":1,"Data":"a\\u003cb\\u003e\\u0026\\"c\\\\ é\\u0001\\u2028","Lower":1,"Upper":2,"Hash":0,"Nonce":0}'
    assert out[3] == '{"Type":0,"Data":"","Lower":0,"Upper":0,"Hash":0,"Nonce":0}\t[Join]'
    # Go skips the field, decodes the rest and returns the error
    assert out[4] == 'TYPEERROR\t{"Type":1,"Data":"","Lower":0,"Upper":0,"Hash":0,"Nonce":0}\t[Request  0 0]'
    assert out[5] == out[4]
    # what Python's json makes of our bytes is the same message back
    assert json.loads(out[2].split("\t")[0])["Data"] == 'a<b>&"c\\ é\u0001\u2028'


def json_lines(mode, lines):
    """p1miner json / lsp-json over raw byte lines -> one output line each
    (bytes: the cases include invalid UTF-8)."""
    r = subprocess.run([MINER, mode], input=b"\n".join(lines) + b"\n", capture_output=True, timeout=60)
    assert r.returncode == 0, r.stderr
    return r.stdout.decode("utf-8").split("\n")[:len(lines)]


def bm(t=0, data="", lo=0, hi=0, h=0, n=0):
    return json.dumps({"Type": t, "Data": data, "Lower": lo, "Upper": hi, "Hash": h, "Nonce": n},
                      separators=(",", ":"), ensure_ascii=False)


def test_json_decode_follows_go_unmarshal():
    """encoding/json.Unmarshal's rules (Go 1.4 decode.go / scanner.go /
    fold.go; gojson.hpp): the whole input is checked first and a syntax
    error changes nothing; a value of the wrong type leaves its field alone
    while the rest is decoded (the miner and client ignore the error,
    miner.go:55, client.go:53, so the partial decode is what they scan);
    strings are unquoted with invalid UTF-8 and lone surrogates as U+FFFD;
    keys fold ASCII case plus U+017F (s) and U+212A (k).  No Go toolchain
    here: the expected values restate those rules; the reference holds no
    fixture for malformed input (parity unpinned for these cases)."""
    cases = [
        # syntax errors: nothing decoded, an error
        (b'{"Type":01}', "ERROR"),
        (b'{"Type":1,}', "ERROR"),
        (b'{"Type":1} x', "ERROR"),
        (b'{"Type":1.}', "ERROR"),
        (b"{'Type':1}", "ERROR"),
        (b'{"Data":"a\tb"}', "ERROR"),              # raw control byte in a string
        (b'{"Data":"\\x"}', "ERROR"),               # unknown escape
        (b'{"Data":"\\u12"}', "ERROR"),
        (b'', "ERROR"),
        (b'[' * 100000, "ERROR"),                   # deep nesting: an error, not a crash
        (b'{"X":' + b'[' * 50000 + b']' * 50000 + b',"Type":2}', bm(2) + "\t[Result 0 0]"),  # skipped
        # type errors: the field is skipped, the rest decoded
        (b'{"Type":1,"Lower":-1,"Upper":10,"Data":"x"}', "TYPEERROR\t" + bm(1, "x", 0, 10) + "\t[Request x 0 10]"),
        (b'{"Type":1,"Lower":1.5,"Upper":2}', "TYPEERROR\t" + bm(1, "", 0, 2) + "\t[Request  0 2]"),
        (b'{"Type":1,"Lower":1e3,"Upper":2}', "TYPEERROR\t" + bm(1, "", 0, 2) + "\t[Request  0 2]"),
        (b'{"Type":1,"Lower":"5","Upper":2}', "TYPEERROR\t" + bm(1, "", 0, 2) + "\t[Request  0 2]"),
        (b'{"Type":"1","Data":"x"}', "TYPEERROR\t" + bm(0, "x") + "\t[Join]"),
        (b'{"Type":1,"Lower":true,"Upper":[1],"Hash":{"a":1},"Nonce":3}',
         "TYPEERROR\t" + bm(1, n=3) + "\t[Request  0 0]"),
        (b'{"Type":9223372036854775808,"Hash":4}', "TYPEERROR\t" + bm(0, h=4) + "\t[Join]"),
        (b'{"Data":true,"Hash":4}', "TYPEERROR\t" + bm(0, h=4) + "\t[Join]"),
        # a number into the string field stops the decode (literalStore's d.error)
        (b'{"Type":1,"Data":5,"Lower":7}', "TYPEERROR\t" + bm(1) + "\t[Request  0 0]"),
        # a non-object top level: a type error (null: no effect, no error)
        (b'[1]', "TYPEERROR\t" + bm() + "\t[Join]"),
        (b'"x"', "TYPEERROR\t" + bm() + "\t[Join]"),
        (b'7', "TYPEERROR\t" + bm() + "\t[Join]"),
        (b' null ', bm() + "\t[Join]"),
        # Go int Type: any int64 decodes
        (b'{"Type":-3,"Hash":1}', bm(-3, h=1) + "\t"),
        (b'{"Type":4294967297}', bm(4294967297) + "\t"),
        # strings: invalid UTF-8 and lone surrogates become U+FFFD
        (b'{"Type":1,"Data":"a\xffb\xe2\x82"}', bm(1, "a\ufffdb\ufffd\ufffd") + "\t[Request a\ufffdb\ufffd\ufffd 0 0]"),
        (b'{"Data":"\\ud800x\\udc00\\ud83d\\ude00"}', bm(0, "\ufffdx\ufffd\U0001F600") + "\t[Join]"),
        (b'{"Data":"\\ud800\\u0041"}', bm(0, "\ufffdA") + "\t[Join]"),
        # keys: case folding, U+017F / U+212A, duplicates (the last wins), nulls
        (b'{"tYPE":1,"dATA":"x","LOWER":2,"upper":3}', bm(1, "x", 2, 3) + "\t[Request x 2 3]"),
        ('{"Ha\u017fh":7,"Type":2}'.encode(), bm(2, h=7) + "\t[Result 7 0]"),
        (b'{"Ha\\u017fh":7,"Type":2}', bm(2, h=7) + "\t[Result 7 0]"),
        (b'{"Hash ":7,"Type":2}', bm(2) + "\t[Result 0 0]"),
        (b'{"Lower":1,"Lower":2,"Type":1}', bm(1, lo=2) + "\t[Request  2 0]"),
        (b'{"Data":null,"Lower":null,"Type":null}', bm() + "\t[Join]"),
    ]
    got = json_lines("json", [c[0] for c in cases])
    for (inp, want), g in zip(cases, got):
        assert g == want, (inp[:80], g, want)


def lm(t=0, c=0, s=0, size=0, payload=None):
    p = "null" if payload is None else '"' + payload + '"'
    return f'{{"Type":{t},"ConnID":{c},"SeqNum":{s},"Size":{size},"Payload":{p}}}'


def test_lsp_json_decode_follows_go_unmarshal():
    """The same rules for lsp.Message (lsp/message.go:16-22): Payload is a
    []byte (base64 string; null -> nil; an array of numbers element-wise;
    bad base64 leaves it unchanged with an error).  The LSP endpoints drop
    every datagram that does not decode error-free (lsp.cpp)."""
    cases = [
        (b'{"Type":1,"ConnID":2,"SeqNum":3,"Size":2,"Payload":"aGk="}', lm(1, 2, 3, 2, "aGk=") + "\t[Data 2 3 hi]"),
        (b'{"Type":1,"Payload":""}', lm(1, payload="") + "\t[Data 0 0 ]"),
        (b'{"Type":1,"Payload":null}', lm(1) + "\t[Data 0 0 ]"),
        (b'{"Type":1,"Payload":"aGk"}', "TYPEERROR\t" + lm(1) + "\t[Data 0 0 ]"),
        (b'{"Type":1,"Payload":"aG\\nk="}', lm(1, payload="aGk=") + "\t[Data 0 0 hi]"),  # \n skipped
        (b'{"Type":1,"Payload":[104,105]}', lm(1, payload="aGk=") + "\t[Data 0 0 hi]"),
        (b'{"Type":1,"Payload":[104,300,"x",105]}', "TYPEERROR\t" + lm(1, payload="aAAAaQ==") + "\t[Data 0 0 h\x00\x00i]"),
        (b'{"Type":1,"Payload":[]}', lm(1, payload="") + "\t[Data 0 0 ]"),
        (b'{"Type":1,"Payload":5,"ConnID":4}', "TYPEERROR\t" + lm(1) + "\t[Data 0 0 ]"),
        (b'{"Type":2,"ConnID":1e2,"SeqNum":-7}', "TYPEERROR\t" + lm(2, 0, -7) + "\t[Ack 0 -7]"),
        (b'{"type":2,"connid":5,"\\u017feqnum":6,"\xc5\xbfize":1}', lm(2, 5, 6, 1) + "\t[Ack 5 6]"),
        (b'{"Type":2,"ConnID":1}}', "ERROR"),
    ]
    got = json_lines("lsp-json", [c[0] for c in cases])
    for (inp, want), g in zip(cases, got):
        assert g == want, (inp, g, want)


def test_cli_usage_errors():
    assert run([]).returncode == 2
    assert run(["scan", "x", "1"]).returncode == 2
    assert run(["scan", "x", "-1", "5"]).returncode == 2


@pytest.mark.gpu
def test_cli_scan_config1():
    # configs[0]: "client 'bradfitz' maxNonce 9999" prints this line (client.go:59-61)
    r = run(["scan", "bradfitz", "0", "9999"])
    assert r.returncode == 0, r.stderr
    assert r.stdout.strip() == "Result 1419516646206828 9898"
    r = run(["hash", "msg", "1"])
    assert r.stdout.strip() == "4754799531757243342"


@pytest.mark.gpu
def test_cli_serve_loop(oracle_mod):
    reqs = [
        {"Type": 0, "Data": "", "Lower": 0, "Upper": 0, "Hash": 0, "Nonce": 0},    # Join: scanned like any line
        {"Type": 1, "Data": "bradfitz", "Lower": 0, "Upper": 9999, "Hash": 0, "Nonce": 0},
        {"Type": 1, "Data": "msg", "Lower": 0, "Upper": 2, "Hash": 0, "Nonce": 0},
        {"Type": 1, "Data": "héllo", "Lower": 10**9 - 3000, "Upper": 10**9 + 3000, "Hash": 0, "Nonce": 0},
        {"Type": 1, "Data": "x", "Lower": 9, "Upper": 3, "Hash": 0, "Nonce": 0},
    ]
    # miner.go:49-67 answers every message it reads: it decodes into a fresh
    # Message (errors ignored) and scans [Lower, Upper] whatever the Type; a
    # line that is not JSON is the request ("", [0, 0]), a line with a type
    # error the fields Go's partial decode kept (here Lower stays 0 and the
    # invalid UTF-8 byte of Data becomes U+FFFD before hashing)
    odd = ['not json', '{"Type":1,"Data":"bradfitz","Lower":-5,"Upper":9999}',
           '{"Type":1,"Data":"a\\udc00b","Lower":"7","Upper":500}']
    stdin = "\n".join(json.dumps(r, ensure_ascii=False) for r in reqs) + "\n" + "\n".join(odd) + "\n"
    r = run(["serve", "--device", "0", "--chunk", "1000"], stdin)  # small chunks: exercises chunking
    assert r.returncode == 0, r.stderr
    res = [json.loads(x) for x in r.stdout.splitlines()]
    assert len(res) == 8 and all(x["Type"] == 2 for x in res)
    want = [oracle_mod.scan(q["Data"], q["Lower"], q["Upper"], threads=8) for q in reqs] + \
        [oracle_mod.scan("", 0, 0), oracle_mod.scan("bradfitz", 0, 9999), oracle_mod.scan("a\ufffdb", 0, 500)]
    assert [(x["Hash"], x["Nonce"]) for x in res] == want
    assert want[4] == (U64_MAX, 0)
    assert want[6] == (1419516646206828, 9898)


def test_lsp_message_wire_format_matches_go():
    # Go encoding/json of lsp.Message (lsp/message.go:16-22): Type, ConnID,
    # SeqNum, Size, Payload ([]byte as padded standard base64, nil as null).
    # Line 1 is the Connect datagram of SURVEY.md Appendix B (what mtest's
    # server accepts); String() follows message.go:51-62.
    lines = [
        '{"Type":0,"ConnID":0,"SeqNum":0,"Size":0,"Payload":null}',
        '{"Type":1,"ConnID":3,"SeqNum":1,"Size":5,"Payload":"aGVsbG8="}',
        '{"type":2,"connid":3,"seqnum":1}',                       # case-insensitive keys, missing fields
        '{"Type":1,"ConnID":1,"SeqNum":2,"Size":0,"Payload":""}',  # empty, non-nil slice
        '{"Type":1,"Payload":"aGVsbG8"}',                          # unpadded base64: Go rejects it
        '{"Type":1,"SeqNum":1.5}',                                 # not an int
        '{"Type":1,"ConnID":-9223372036854775808,"SeqNum":9223372036854775807,"Payload":"w6k="}',
        '{"Type":1,"ConnID":9223372036854775808}',                 # int64 overflow
    ]
    out = run(["lsp-json"], "\n".join(lines) + "\n").stdout.split("\n")
    assert out[0] == lines[0] + "\t[Connect 0 0]"
    assert out[1] == lines[1] + "\t[Data 3 1 hello]"
    assert out[2] == '{"Type":2,"ConnID":3,"SeqNum":1,"Size":0,"Payload":null}\t[Ack 3 1]'
    assert out[3] == lines[3] + "\t[Data 1 2 ]"
    # type errors: the field keeps its value, the rest is decoded
    assert out[4] == 'TYPEERROR\t{"Type":1,"ConnID":0,"SeqNum":0,"Size":0,"Payload":null}\t[Data 0 0 ]'
    assert out[5] == out[4] and out[7] == out[4]
    assert out[6].split("\t")[0] == \
        '{"Type":1,"ConnID":-9223372036854775808,"SeqNum":9223372036854775807,"Size":0,"Payload":"w6k="}'


def test_lsp_framing_of_bitcoin_messages():
    # miner.go:21,66: client.Write(json.Marshal(msg)) -> one LSP Data datagram
    # whose Payload is the bitcoin.Message JSON and Size its length.
    import base64

    msgs = ['{"Type":0,"Data":"","Lower":0,"Upper":0,"Hash":0,"Nonce":0}',
            '{"Type":2,"Data":"","Lower":0,"Upper":0,"Hash":1419516646206828,"Nonce":9898}',
            '{"Type":1,"Data":"~~~???","Lower":7,"Upper":8,"Hash":0,"Nonce":0}']  # '+' and '/' in base64
    wrapped = run(["lsp-wrap", "7", "1"], "\n".join(msgs) + "\n").stdout.strip().split("\n")
    for i, (w, m) in enumerate(zip(wrapped, msgs)):
        d = json.loads(w)
        assert list(d) == ["Type", "ConnID", "SeqNum", "Size", "Payload"]
        assert (d["Type"], d["ConnID"], d["SeqNum"], d["Size"]) == (1, 7, 1 + i, len(m))
        assert base64.b64decode(d["Payload"]).decode() == m
    assert "+" in wrapped[2] and "/" in wrapped[2]
    back = run(["lsp-unwrap"], "\n".join(wrapped) + "\n").stdout.strip().split("\n")
    assert back == msgs
