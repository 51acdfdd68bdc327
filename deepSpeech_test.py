#!/usr/bin/env python3
"""CLI-compatible entrypoint (reference: src/deepSpeech_test.py) -> deepspeech_amd.test.

The platform environment (reference src/setenvs.py) is applied BEFORE torch is imported.
"""
import sys

from deepspeech_amd.utils.setenvs import setenvs

setenvs(sys.argv)

from deepspeech_amd.test import main  # noqa: E402

if __name__ == "__main__":
    sys.exit(main())
