module github.com/jflyup/ugo/ugofec

go 1.20
