"""flexflow_amd.models"""
