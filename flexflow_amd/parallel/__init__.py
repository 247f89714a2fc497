"""flexflow_amd.parallel"""
