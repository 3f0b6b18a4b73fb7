"""Global image descriptors (gtsfm/frontend/global_descriptor/)."""
