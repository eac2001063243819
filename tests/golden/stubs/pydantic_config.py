"""Offline stand-in for the `pydantic_config` git dependency (requirements.txt:7 of the
reference). Only `BaseConfig` is needed to import the reference's hot-path modules; the CLI
parser is never used by the fixture capture and raises if called."""
from pydantic import BaseModel, ConfigDict


class BaseConfig(BaseModel):
    model_config = ConfigDict(extra="forbid")


def parse_argv(*args, **kwargs):
    raise RuntimeError("parse_argv is not available offline")
