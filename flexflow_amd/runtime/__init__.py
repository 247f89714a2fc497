"""flexflow_amd.runtime"""
