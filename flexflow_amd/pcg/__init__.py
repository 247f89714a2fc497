"""flexflow_amd.pcg"""
