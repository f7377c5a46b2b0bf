"""empty import-time stub (test-only); HDF5 I/O is out of scope"""
