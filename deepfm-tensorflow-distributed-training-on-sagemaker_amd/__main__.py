"""``python -m hipfm`` == the reference's ``python DeepFM-*.py`` (flag-compatible)."""
from .cli import main

main()
