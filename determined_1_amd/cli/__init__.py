"""``det`` command line (reference ``cli/determined_cli/``)."""
