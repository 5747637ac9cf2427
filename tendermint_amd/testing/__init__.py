"""Synthetic-workload factories (the analogue of the reference's
internal/test/factory).  Signing happens here, on the host, only to build
inputs; nothing in this subpackage verifies anything."""
