"""``python -m uncertaintyquantification_sleepapnea_1dcnn_amd <command>`` (see cli/commands.py)."""
import sys

from .cli.commands import main

sys.exit(main())
