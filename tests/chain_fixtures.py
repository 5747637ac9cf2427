"""host.* light-client objects -> oracle/light_ref.py objects, and the
oracle's light drivers over them (the checker for tendermint_amd/chains.py)."""
import light_ref as L


def block_id(b):
    return L.BlockID(b.hash, b.psh_total, b.psh_hash)


def header(h):
    return L.Header(version_block=h.version_block, version_app=h.version_app, chain_id=h.chain_id, height=h.height,
                    time_ns=h.time[0] * L.NS + h.time[1], last_block_id=block_id(h.last_block_id),
                    last_commit_hash=h.last_commit_hash, data_hash=h.data_hash, validators_hash=h.validators_hash,
                    next_validators_hash=h.next_validators_hash, consensus_hash=h.consensus_hash,
                    app_hash=h.app_hash, last_results_hash=h.last_results_hash, evidence_hash=h.evidence_hash,
                    proposer_address=h.proposer_address)


def commit(c):
    return L.Commit(c.height, c.round, block_id(c.block_id),
                    [L.CommitSig(s.block_id_flag, s.validator_address, s.timestamp[0] * L.NS + s.timestamp[1],
                                 s.signature) for s in c.signatures])


def signed_header(sh):
    return L.SignedHeader(header(sh.header), commit(sh.commit))


def valset(vs):
    return L.ValidatorSet([L.Validator(v.address, v.pub_key, v.voting_power, v.key_kind, v.proposer_priority)
                           for v in vs.validators])


class OracleBlocks:
    """Memoised conversion (one oracle object per host object)."""

    def __init__(self):
        self.m = {}

    def __call__(self, lb):
        if id(lb) not in self.m:
            self.m[id(lb)] = (lb, L.LightBlock(signed_header(lb.signed_header), valset(lb.vals)))
        return self.m[id(lb)][1]
