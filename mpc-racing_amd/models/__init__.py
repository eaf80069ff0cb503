"""Vehicle constants and state record used by the drop-in controller (reference ``models/``)."""
