"""Shared utilities: validation, logging/request ids, retry."""
