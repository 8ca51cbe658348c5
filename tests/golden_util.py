import json
import os

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


def load(group):
    with open(os.path.join(GOLDEN, group + ".json")) as f:
        return json.load(f)


def case_id(c):
    return "%s|%s" % (c.get("source", "").rsplit("/", 1)[-1], c.get("test", c.get("q", ""))[:60])
