"""On-disk caches for the front-end plugins (reference gtsfm/frontend/cacher/)."""
