#!/usr/bin/env python3
"""CLI-compatible entrypoint (reference: src/deepSpeech_test.py) -> deepspeech_amd.test."""
import sys

from deepspeech_amd.test import main

if __name__ == "__main__":
    sys.exit(main())
