"""Nebula (asynchronous tiered checkpoint service) configuration (reference `nebula/`). The service itself is an
external Azure component; this framework's asynchronous writer is `runtime/checkpoint_engine.AsyncCheckpointEngine`,
selected by the same `nebula.enabled` key."""
