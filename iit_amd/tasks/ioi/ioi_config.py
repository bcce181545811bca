"""IOI vocabulary data: names, templates and nouns (synthetic, offline).

Only ``NAMES`` of the reference's 976-line ``ioi_config.py`` is used by its
pipeline (``/root/reference/iit/tasks/ioi/__init__.py:2``,
``/root/reference/train_ioi.py:7``); the rest is dead code and is not rebuilt.
The list below is this framework's own (common single-token first names).
"""

NAMES = [
    "Aaron", "Adam", "Alan", "Alex", "Alice", "Amanda", "Amy", "Andrew", "Angela", "Anna",
    "Anthony", "Arthur", "Austin", "Barbara", "Ben", "Betty", "Bill", "Bob", "Brad", "Brian",
    "Bruce", "Carl", "Carol", "Charles", "Chris", "Claire", "Colin", "Craig", "Dan", "Daniel",
    "David", "Dean", "Diana", "Donna", "Doug", "Edward", "Elena", "Emily", "Emma", "Eric",
    "Frank", "Fred", "Gary", "George", "Grace", "Greg", "Hannah", "Harry", "Helen", "Henry",
    "Ian", "Jack", "Jacob", "James", "Jane", "Jason", "Jeff", "Jennifer", "Jessica", "Jim",
    "Joe", "John", "Jordan", "Joseph", "Julia", "Karen", "Kate", "Kevin", "Kyle", "Laura",
    "Lisa", "Louis", "Lucy", "Marco", "Maria", "Mark", "Martin", "Mary", "Matt", "Michael",
    "Mike", "Nancy", "Neil", "Nick", "Oliver", "Paul", "Peter", "Rachel", "Ray", "Richard",
    "Robert", "Rose", "Ryan", "Sam", "Sarah", "Scott", "Sophie", "Steve", "Tom", "Victoria",
]

TEMPLATES = [
    "Then, [B] and [A] went to the [LOCATION]. [A] gave the [OBJECT] to [B]",
    "Then, [A] and [B] went to the [LOCATION]. [B] gave the [OBJECT] to [A]",
    "Then, [A] and [B] went to the [LOCATION]. [A] gave the [OBJECT] to [B]",
    "Then, [B] and [A] went to the [LOCATION]. [B] gave the [OBJECT] to [A]",
]

NOUNS = {
    "LOCATION": ["store", "market"],
    "OBJECT": ["milk", "eggs", "bread"],
}


def vocabulary_words():
    """Every piece the IOI prompts can contain, in a fixed registration order."""
    words = ["Then", ",", ".", " and", " went", " to", " the", " gave"]
    for lst in NOUNS.values():
        words += [" " + w for w in lst]
    words += [" " + n for n in NAMES]
    return words
