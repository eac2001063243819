"""Offline stand-in for python-dotenv."""


def load_dotenv(*args, **kwargs):
    return False
