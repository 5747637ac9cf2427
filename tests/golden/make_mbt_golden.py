"""Convert the reference's model-based light-client fixtures
(/root/reference/light/mbt/json/*.json, driven by light/mbt/driver_test.go:
18-86) into tests/golden/mbt_light.json.

Data only: headers, commits (ed25519 signatures), validator sets, trusting
period, `now` and the expected light.Verify verdict of every input, re-encoded
with hex bytes and (seconds, nanos) times so the tests need neither the
reference tree nor a Go-style JSON decoder.  Run in the build container (the
reference is absent on the GPU box):

    python tests/golden/make_mbt_golden.py
"""
import base64
import glob
import json
import os
import re

SRC = "/root/reference/light/mbt/json"
OUT = os.path.join(os.path.dirname(os.path.abspath(__file__)), "mbt_light.json")


def days_from_civil(y, m, d):
    y -= m <= 2
    era = (y if y >= 0 else y - 399) // 400
    yoe = y - era * 400
    doy = (153 * (m + (-3 if m > 2 else 9)) + 2) // 5 + d - 1
    doe = yoe * 365 + yoe // 4 - yoe // 100 + doy
    return era * 146097 + doe - 719468


def rfc3339(s):
    """RFC 3339 UTC timestamp -> [seconds since epoch, nanos]."""
    if s is None:
        return [-62135596800, 0]
    m = re.fullmatch(r"(\d{4})-(\d\d)-(\d\d)T(\d\d):(\d\d):(\d\d)(?:\.(\d{1,9}))?Z", s)
    assert m, s
    y, mo, d, hh, mm, ss = (int(m.group(i)) for i in range(1, 7))
    nanos = int((m.group(7) or "0").ljust(9, "0"))
    return [days_from_civil(y, mo, d) * 86400 + hh * 3600 + mm * 60 + ss, nanos]


def hx(s):
    return (s or "").lower()


def block_id(b):
    if b is None:
        return {"hash": "", "psh_total": 0, "psh_hash": ""}
    parts = b.get("parts") or b.get("part_set_header") or {}
    return {"hash": hx(b.get("hash")), "psh_total": int(parts.get("total") or 0), "psh_hash": hx(parts.get("hash"))}


def header(h):
    return {
        "version_block": int(h["version"]["block"]), "version_app": int(h["version"].get("app") or 0),
        "chain_id": h["chain_id"], "height": int(h["height"]), "time": rfc3339(h["time"]),
        "last_block_id": block_id(h.get("last_block_id")),
        **{k: hx(h.get(k)) for k in ("last_commit_hash", "data_hash", "validators_hash", "next_validators_hash",
                                     "consensus_hash", "app_hash", "last_results_hash", "evidence_hash",
                                     "proposer_address")},
    }


def commit(c):
    sigs = []
    for s in c["signatures"]:
        sigs.append({"flag": int(s["block_id_flag"]), "address": hx(s.get("validator_address")),
                     "time": rfc3339(s.get("timestamp")),
                     "signature": base64.b64decode(s["signature"]).hex() if s.get("signature") else ""})
    return {"height": int(c["height"]), "round": int(c["round"]), "block_id": block_id(c["block_id"]),
            "signatures": sigs}


def valset(vs):
    out = []
    for v in vs["validators"]:
        assert v["pub_key"]["type"] == "tendermint/PubKeyEd25519", v["pub_key"]["type"]
        out.append({"address": hx(v["address"]), "pub_key": base64.b64decode(v["pub_key"]["value"]).hex(),
                    "voting_power": int(v["voting_power"]), "proposer_priority": int(v.get("proposer_priority") or 0)})
    return out


def signed_header(sh):
    return {"header": header(sh["header"]), "commit": commit(sh["commit"])}


def main():
    cases = []
    for path in sorted(glob.glob(os.path.join(SRC, "*.json"))):
        with open(path) as f:
            tc = json.load(f)
        ini = tc["initial"]
        case = {"file": "light/mbt/json/" + os.path.basename(path), "description": tc["description"],
                "initial": {"signed_header": signed_header(ini["signed_header"]),
                            "next_validator_set": valset(ini["next_validator_set"]),
                            "trusting_period_ns": int(ini["trusting_period"]), "now": rfc3339(ini["now"])},
                "input": []}
        for inp in tc["input"]:
            b = inp["block"]
            case["input"].append({"signed_header": signed_header(b["signed_header"]),
                                  "validator_set": valset(b["validator_set"]),
                                  "next_validator_set": valset(b["next_validator_set"]),
                                  "now": rfc3339(inp["now"]), "verdict": inp["verdict"]})
        cases.append(case)
    with open(OUT, "w") as f:
        json.dump({"source": "AnastasiaBelenkii/tendermint light/mbt/json (model-based tests, tendermint-rs generated)",
                   "driver": "light/mbt/driver_test.go:18-86 (light.Verify, maxClockDrift 1s, trust level 1/3)",
                   "cases": cases}, f, indent=1)
    print(f"{OUT}: {len(cases)} cases, {sum(len(c['input']) for c in cases)} inputs")


if __name__ == "__main__":
    main()
