"""Host-side mirror of the reference's ``types`` package for the hot path
(commit layout, sign-bytes, VerifyCommit family)."""
