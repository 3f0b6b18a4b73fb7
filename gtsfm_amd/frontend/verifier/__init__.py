"""gtsfm_amd package."""
