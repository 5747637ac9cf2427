"""Loader for tests/golden/mbt_light.json (the reference's light/mbt/json
model-based fixtures, converted by tests/golden/make_mbt_golden.py) into the
oracle's types (oracle/light_ref.py)."""
import json
import os

import light_ref as L

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "mbt_light.json")
MAX_CLOCK_DRIFT_NS = 1_000_000_000  # light/mbt/driver_test.go:53
TRUST_LEVEL = (1, 3)                # light.DefaultTrustLevel, light/verifier.go:16
VERDICT_KIND = {"SUCCESS": (L.OK,), "NOT_ENOUGH_TRUST": (L.CANT_TRUST,),
                "INVALID": (L.INVALID_HEADER, L.OLD_HEADER_EXPIRED)}


def _ns(t):
    return t[0] * L.NS + t[1]


def _b(h):
    return bytes.fromhex(h)


def block_id(d):
    return L.BlockID(_b(d["hash"]), d["psh_total"], _b(d["psh_hash"]))


def header(d):
    return L.Header(version_block=d["version_block"], version_app=d["version_app"], chain_id=d["chain_id"],
                    height=d["height"], time_ns=_ns(d["time"]), last_block_id=block_id(d["last_block_id"]),
                    **{k: _b(d[k]) for k in ("last_commit_hash", "data_hash", "validators_hash",
                                             "next_validators_hash", "consensus_hash", "app_hash",
                                             "last_results_hash", "evidence_hash", "proposer_address")})


def commit(d):
    return L.Commit(d["height"], d["round"], block_id(d["block_id"]),
                    [L.CommitSig(s["flag"], _b(s["address"]), _ns(s["time"]), _b(s["signature"]))
                     for s in d["signatures"]])


def signed_header(d):
    return L.SignedHeader(header(d["header"]), commit(d["commit"]))


def valset(d):
    return L.ValidatorSet([L.Validator(_b(v["address"]), _b(v["pub_key"]), v["voting_power"], L.KIND_ED25519,
                                       v["proposer_priority"]) for v in d])


def load_cases():
    with open(GOLDEN) as f:
        data = json.load(f)
    out = []
    for c in data["cases"]:
        ini = c["initial"]
        case = {"file": c["file"], "trusted": signed_header(ini["signed_header"]),
                "trusted_next_vals": valset(ini["next_validator_set"]),
                "trusting_period_ns": ini["trusting_period_ns"], "inputs": []}
        for inp in c["input"]:
            case["inputs"].append({"signed_header": signed_header(inp["signed_header"]),
                                   "vals": valset(inp["validator_set"]),
                                   "next_vals": valset(inp["next_validator_set"]),
                                   "now_ns": _ns(inp["now"]), "verdict": inp["verdict"]})
        out.append(case)
    return out


def run_driver(case, verify):
    """light/mbt/driver_test.go:42-81: Verify every input against the current
    trusted (header, next vals); advance on success.  `verify(trusted,
    trusted_next_vals, untrusted, untrusted_vals, trusting_period_ns, now_ns,
    drift_ns, trust)` returns None or an object with .kind and .text.
    Yields (input, result)."""
    trusted, tnext = case["trusted"], case["trusted_next_vals"]
    for inp in case["inputs"]:
        r = verify(trusted, tnext, inp["signed_header"], inp["vals"], case["trusting_period_ns"], inp["now_ns"],
                   MAX_CLOCK_DRIFT_NS, TRUST_LEVEL)
        yield inp, r
        if r is None:
            trusted, tnext = inp["signed_header"], inp["next_vals"]


# ---------------------------------------------------------------- host (product) types
def _host():
    from tendermint_amd import host as H
    return H


def host_block_id(d):
    H = _host()
    return H.BlockID(_b(d["hash"]), d["psh_total"], _b(d["psh_hash"]))


def host_header(d):
    H = _host()
    return H.Header(chain_id=d["chain_id"], height=d["height"], time=tuple(d["time"]),
                    last_block_id=host_block_id(d["last_block_id"]), version_block=d["version_block"],
                    version_app=d["version_app"],
                    **{k: _b(d[k]) for k in ("last_commit_hash", "data_hash", "validators_hash",
                                             "next_validators_hash", "consensus_hash", "app_hash",
                                             "last_results_hash", "evidence_hash", "proposer_address")})


def host_commit(d):
    H = _host()
    return H.Commit(d["height"], d["round"], host_block_id(d["block_id"]),
                    [H.CommitSig(s["flag"], _b(s["address"]), tuple(s["time"]), _b(s["signature"]))
                     for s in d["signatures"]])


def host_signed_header(d):
    H = _host()
    return H.SignedHeader(host_header(d["header"]), host_commit(d["commit"]))


def host_valset(d):
    H = _host()
    return H.ValidatorSet([H.Validator(_b(v["address"]), _b(v["pub_key"]), v["voting_power"], H.TMV_KIND_ED25519,
                                       v["proposer_priority"]) for v in d], proposer_index=-1)


def load_host_cases():
    with open(GOLDEN) as f:
        data = json.load(f)
    out = []
    for c in data["cases"]:
        ini = c["initial"]
        out.append({"file": c["file"], "trusted": host_signed_header(ini["signed_header"]),
                    "trusted_next_vals": host_valset(ini["next_validator_set"]),
                    "trusting_period_ns": ini["trusting_period_ns"],
                    "inputs": [{"signed_header": host_signed_header(i["signed_header"]),
                                "vals": host_valset(i["validator_set"]),
                                "next_vals": host_valset(i["next_validator_set"]), "now": tuple(i["now"]),
                                "verdict": i["verdict"]} for i in c["input"]]})
    return out


def run_host_driver(case, verify_many):
    """driver_test.go:42-81 through the host layer: verify_many(list of
    host.LightJob) -> [(kind, text)].  Yields (input, (kind, text))."""
    H = _host()
    trusted, tnext = case["trusted"], case["trusted_next_vals"]
    for inp in case["inputs"]:
        job = H.LightJob(trusted, tnext, inp["signed_header"], inp["vals"], case["trusting_period_ns"], inp["now"],
                         MAX_CLOCK_DRIFT_NS, TRUST_LEVEL)
        r = verify_many([job])[0]
        yield inp, r
        if r[0] == H.LIGHT_OK:
            trusted, tnext = inp["signed_header"], inp["next_vals"]
