#!/usr/bin/env python3
"""CLI-compatible entrypoint (reference: src/deepSpeech_train.py) -> deepspeech_amd.train."""
import sys

from deepspeech_amd.train import main

if __name__ == "__main__":
    sys.exit(main())
