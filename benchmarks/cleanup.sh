#!/usr/bin/env bash
cd "$(dirname "$0")"
rm -f ./*.dat ./*.png
