"""empty import-time stub (test-only); sed_eval metrics are out of scope"""
