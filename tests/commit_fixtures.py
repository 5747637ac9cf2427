"""Commit / validator-set builders for the commit-verification tests, in the
shape of the reference's fixtures (types/vote_set_test.go:588-632
randVoteSet / randValidatorPrivValSet, types/test_util.go:11-37
makeExtCommit, types/block_test.go:225-239 makeBlockID).

scheme "fake": test-double signatures SHA-512(pk || 0^32 || M) checked by
tests/native/commit_check.cpp (CPU, no crypto); "ed25519" / "sr25519": real
signatures for the GPU path."""
import ctypes
import hashlib
import os

from tendermint_amd import host as H
from tendermint_amd.types.canonical import (BlockID as PyBlockID, PartSetHeader, Timestamp, vote_sign_bytes,
                                            PRECOMMIT_TYPE)

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
# TMV_COMMITCHECK_SO: another build of the harness (the ASan/UBSan one, tests/test_sanitizers.py)
CHECK_SO = os.environ.get("TMV_COMMITCHECK_SO", os.path.join(REPO, "oracle", "_build", "libcommitcheck.so"))


def make_block_id(hash_: bytes, total: int, psh: bytes) -> H.BlockID:
    return H.BlockID(hash_.ljust(32, b"\0")[:32], total, psh.ljust(32, b"\0")[:32])


def random_block_id(seed: int) -> H.BlockID:
    r = hashlib.sha256(b"bid %d" % seed).digest()
    return H.BlockID(r, 1 + seed % 1000, hashlib.sha256(r).digest())


class Signer:
    def __init__(self, scheme: str, i: int, tag: str = "key"):
        self.scheme = scheme
        secret = f"{tag}: {i:x}".encode()
        if scheme == "ed25519":
            from tendermint_amd.testing._openssl import Ed25519Signer
            self._s = Ed25519Signer(hashlib.sha256(secret).digest())
            self.pub_key = self._s.public_key
            self.kind = H.TMV_KIND_ED25519
        elif scheme == "sr25519":
            from tendermint_amd.testing.sr25519_factory import Sr25519Signer, mini_from_secret
            self._s = Sr25519Signer(mini_from_secret(secret))
            self.pub_key = self._s.public_key
            self.kind = H.TMV_KIND_SR25519
        else:
            self.pub_key = hashlib.sha256(b"fake " + secret).digest()
            self.kind = H.TMV_KIND_ED25519
        self.address = hashlib.sha256(self.pub_key).digest()[:20]  # crypto.AddressHash

    def sign(self, msg: bytes) -> bytes:
        if self.scheme in ("ed25519", "sr25519"):
            return self._s.sign(msg)
        return hashlib.sha512(self.pub_key + bytes(32) + msg).digest()


def rand_val_set(scheme: str, n: int, power: int, tag: str = "key"):
    signers = sorted((Signer(scheme, i, tag) for i in range(n)), key=lambda s: s.address)
    vals = H.ValidatorSet([H.Validator(s.address, s.pub_key, power, s.kind) for s in signers], proposer_index=0)
    return vals, signers


def sign_commit_sig(signer, chain_id, height, round_, block_id: H.BlockID, flag, ts):
    bid = None
    if flag == H.BLOCK_ID_FLAG_COMMIT:
        bid = PyBlockID(block_id.hash, PartSetHeader(block_id.psh_total, block_id.psh_hash))
    msg = vote_sign_bytes(chain_id, PRECOMMIT_TYPE, height, round_, bid, Timestamp(*ts))
    return H.CommitSig(flag, signer.address, ts, signer.sign(msg))


def make_commit(signers, chain_id, height, round_, block_id, ts0=(1577836800, 0)):
    """makeExtCommit: every validator signs a precommit for block_id."""
    sigs = [sign_commit_sig(s, chain_id, height, round_, block_id, H.BLOCK_ID_FLAG_COMMIT,
                            (ts0[0], ts0[1] + i * 1000)) for i, s in enumerate(signers)]
    return H.Commit(height, round_, block_id, sigs)


class FakeBackend:
    """Runs the C++ commit verifier (tm_types.h) with the test-double scheme."""

    def __init__(self):
        import subprocess
        if "TMV_COMMITCHECK_SO" not in os.environ:
            subprocess.run(["make", "-s", "-C", os.path.join(REPO, "tests", "native")], check=True)
        self.L = ctypes.CDLL(CHECK_SO)
        self.L.commitcheck_verify_commit.argtypes = [ctypes.c_int, ctypes.c_char_p, ctypes.POINTER(H.CValidator),
                                                     ctypes.c_uint32, ctypes.c_int32, ctypes.POINTER(H.CBlockID),
                                                     ctypes.c_int64, ctypes.POINTER(H.CCommit), ctypes.c_int64,
                                                     ctypes.c_int64, ctypes.c_char_p, ctypes.c_size_t]
        self.scheme = "fake"

    def _call(self, mode, chain_id, vals, block_id, height, commit, trust=(0, 1)):
        fn = lambda _h, *a: self.L.commitcheck_verify_commit(*a)  # noqa: E731
        return H._commit_call(fn, None, mode, chain_id, vals, block_id, height, commit, trust)

    def verify_commit(self, chain_id, vals, block_id, height, commit):
        return self._call(H.MODE_FULL, chain_id, vals, block_id, height, commit)

    def verify_commit_light(self, chain_id, vals, block_id, height, commit):
        return self._call(H.MODE_LIGHT, chain_id, vals, block_id, height, commit)

    def verify_commit_light_trusting(self, chain_id, vals, commit, trust=(1, 3)):
        return self._call(H.MODE_LIGHT_TRUSTING, chain_id, vals, None, 0, commit, trust)

    def batches_made(self):
        return ctypes.c_int.in_dll(self.L, "commitcheck_backend_calls").value

    def real_signatures(self, on: bool):
        """Switch the test double to the C oracle's ed25519 / sr25519 verification."""
        self.L.commitcheck_set_real_signatures(1 if on else 0)

    def light_verify_many(self, jobs):
        L = self.L
        if not getattr(L, "_light", False):
            L.commitcheck_light_verify_many.argtypes = [ctypes.POINTER(H.CLightJob), ctypes.c_uint32,
                                                        ctypes.POINTER(ctypes.c_int32), ctypes.c_char_p,
                                                        ctypes.c_size_t]
            L.commitcheck_header_hashes.argtypes = [ctypes.POINTER(H.CHeader), ctypes.c_uint32,
                                                    ctypes.POINTER(ctypes.c_uint8), ctypes.POINTER(ctypes.c_uint8)]
            L._light = True
        fn = lambda _h, *a: L.commitcheck_light_verify_many(*a)  # noqa: E731
        return H.run_light_jobs(fn, None, H.PreparedLightJobs(jobs))

    def header_hashes(self, headers):
        self.light_verify_many([])  # argtypes
        fn = lambda _h, *a: self.L.commitcheck_header_hashes(*a)  # noqa: E731
        return H.header_hashes_call(fn, None, headers)


class GpuBackend:
    def __init__(self, ctx, scheme="ed25519"):
        self.ctx, self.scheme = ctx, scheme

    def verify_commit(self, chain_id, vals, block_id, height, commit):
        return H.verify_commit(self.ctx, chain_id, vals, block_id, height, commit)

    def verify_commit_light(self, chain_id, vals, block_id, height, commit):
        return H.verify_commit_light(self.ctx, chain_id, vals, block_id, height, commit)

    def verify_commit_light_trusting(self, chain_id, vals, commit, trust=(1, 3)):
        return H.verify_commit_light_trusting(self.ctx, chain_id, vals, commit, trust)


def fake_verify_commits(backend: "FakeBackend", jobs):
    L = backend.L
    if not getattr(L, "_many", False):
        L.commitcheck_verify_commits.argtypes = [ctypes.POINTER(H.CCommitJob), ctypes.c_uint32,
                                                 ctypes.POINTER(ctypes.c_int32), ctypes.c_char_p, ctypes.c_size_t]
        L._many = True
    pj = H.PreparedJobs(jobs)
    L.commitcheck_verify_commits(pj.arr, pj.n, pj.results, pj.errs, pj.stride)
    return pj.decode()


def random_jobs(scheme: str, n_jobs: int, seed: int):
    """Random commit checks covering every branch: sizes 1..9, absent / nil /
    commit flags, corrupted signatures, wrong block IDs / heights, all three
    modes, shared commits (checked twice, like blocksync)."""
    import random
    rng = random.Random(seed)
    jobs = []
    pool = {}
    for j in range(n_jobs):
        nv = rng.randint(1, 9)
        if nv not in pool:
            pool[nv] = rand_val_set(scheme, nv, rng.randint(1, 50), tag=f"r{nv}")
        vals, signers = pool[nv]
        vals = H.ValidatorSet([H.Validator(v.address, v.pub_key, rng.randint(1, 30), v.key_kind)
                               for v in vals.validators], 0)
        height = rng.randint(1, 5)
        bid = random_block_id(rng.randint(0, 3))
        sigs = []
        for i, s in enumerate(signers):
            r = rng.random()
            if r < 0.15:
                sigs.append(H.CommitSig())
                continue
            flag = H.BLOCK_ID_FLAG_NIL if r < 0.3 else H.BLOCK_ID_FLAG_COMMIT
            chain = "chain" if rng.random() > 0.1 else "other"
            sigs.append(sign_commit_sig(s, chain, height, 0, bid, flag, (1577836800 + i, rng.randrange(10**9))))
        commit = H.Commit(height, 0, bid, sigs)
        mode = rng.choice([H.MODE_FULL, H.MODE_LIGHT, H.MODE_LIGHT_TRUSTING])
        want_bid = bid if rng.random() > 0.1 else random_block_id(9)
        want_h = height if rng.random() > 0.1 else height + 1
        jobs.append(H.CommitJob(mode, "chain", vals, want_bid, want_h, commit, (rng.randint(1, 2), 3)))
        if rng.random() < 0.3:  # same commit checked again (blocksync: light then full)
            jobs.append(H.CommitJob(H.MODE_FULL, "chain", vals, want_bid, want_h, commit))
    return jobs


def single_result(backend, jb):
    if jb.mode == H.MODE_FULL:
        return backend.verify_commit(jb.chain_id, jb.vals, jb.block_id, jb.height, jb.commit)
    if jb.mode == H.MODE_LIGHT:
        return backend.verify_commit_light(jb.chain_id, jb.vals, jb.block_id, jb.height, jb.commit)
    return backend.verify_commit_light_trusting(jb.chain_id, jb.vals, jb.commit, jb.trust)
