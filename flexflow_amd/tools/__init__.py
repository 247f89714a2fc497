"""Command-line tools (reference tools/): protobuf_to_json, substitutions_to_dot."""
