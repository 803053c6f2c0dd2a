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
        '{"Type":1,"Lower":-1}',                                  # negative uint64 rejected
        '{"Type":1,"Upper":18446744073709551616}',                # overflow rejected
    ]
    out = run(["json"], "\n".join(lines) + "\n").stdout.split("\n")
    assert out[0] == lines[0] + "\t[Request bradfitz 0 9999]"
    assert out[1] == '{"Type":2,"Data":"","Lower":0,"Upper":0,"Hash":18446744073709551615,"Nonce":5}' \
                     "\t[Result 18446744073709551615 5]"
    assert out[2].split("\t")[0] == \
        '{"Type":1,"Data":"a\\u003cb\\u003e\\u0026\\"c\\\\ é\\u0001\\u2028","Lower":1,"Upper":2,"Hash":0,"Nonce":0}'
    assert out[3] == '{"Type":0,"Data":"","Lower":0,"Upper":0,"Hash":0,"Nonce":0}\t[Join]'
    assert out[4] == "ERROR" and out[5] == "ERROR"
    # what Python's json makes of our bytes is the same message back
    assert json.loads(out[2].split("\t")[0])["Data"] == 'a<b>&"c\\ é\u0001\u2028'


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
    # miner.go:49-67 answers every message it reads: it decodes into a zero
    # Message (errors ignored) and scans [Lower, Upper] whatever the Type; an
    # undecodable line is the request ("", [0, 0])
    stdin = "\n".join(json.dumps(r, ensure_ascii=False) for r in reqs) + "\nnot json\n"
    r = run(["serve", "--device", "0", "--chunk", "1000"], stdin)  # small chunks: exercises chunking
    assert r.returncode == 0, r.stderr
    res = [json.loads(x) for x in r.stdout.splitlines()]
    assert len(res) == 6 and all(x["Type"] == 2 for x in res)
    want = [oracle_mod.scan(q["Data"], q["Lower"], q["Upper"], threads=8) for q in reqs] + [oracle_mod.scan("", 0, 0)]
    assert [(x["Hash"], x["Nonce"]) for x in res] == want
    assert want[-2] == (U64_MAX, 0)


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
    assert out[4] == "ERROR" and out[5] == "ERROR" and out[7] == "ERROR"
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
