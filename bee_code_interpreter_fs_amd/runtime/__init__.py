"""Sandbox runtime: zygote, single-use workers, in-sandbox patches, deps."""
