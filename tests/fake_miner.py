"""TEST DOUBLE for p1server's CPU tests: a miner process speaking the same
newline-delimited bitcoin.Message JSON as `p1miner serve`, answering with the
oracle (no GPU).  FAKE_DIE_AFTER=n makes it exit without answering its
(n+1)-th request (a lost miner)."""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import oracle  # noqa: E402

die_after = int(os.environ.get("FAKE_DIE_AFTER", "-1"))
seen = 0
for line in sys.stdin:
    req = json.loads(line)
    if req.get("Type") != 1:
        continue
    if seen == die_after:
        sys.exit(3)
    seen += 1
    h, n = oracle.scan(req["Data"].encode("utf-8"), req["Lower"], req["Upper"])
    sys.stdout.write(json.dumps({"Type": 2, "Data": "", "Lower": 0, "Upper": 0, "Hash": h, "Nonce": n}) + "\n")
    sys.stdout.flush()
