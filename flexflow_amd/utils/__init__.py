"""flexflow_amd.utils"""
